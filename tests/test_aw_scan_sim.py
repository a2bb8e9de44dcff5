"""aw_scan's pruning (csrc/sbr_baseline.hip), restated in tools/aw_scan_sim.py, returns the
exhaustive AW_max bit for bit with the shipped run bounds and with each knot's own AW_OUT bound
(SBR_AW_OWN), and the own bound needs fewer exact evaluations (CPU, oracle knots; the GPU A/B
found the kernel slower with it all the same, so SBR_AW_OWN is off: profiles/experiments/r05_d_*)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
import aw_scan_sim  # noqa: E402


def test_own_bound_same_max_fewer_evaluations(capsys):
    aw_scan_sim.main(ncol=8, ustride=32)  # asserts max == the oracle's exhaustive AW_max per point
    out = capsys.readouterr().out
    shipped = float(out.split("shipped ")[1].split(",")[0])
    own = float(out.split("own-knot bound ")[1].split(",")[0])
    assert own < 0.8 * shipped
