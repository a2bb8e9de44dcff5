"""Diagnostic only (not a bench line): the default bench with kernel-timing events disabled in
the timed region, to measure what the per-launch event markers cost the wall-clock step.
The kernel times it prints are placeholders."""
import sys
sys.path.insert(0, ".")
import bench  # noqa: E402
import sbr  # noqa: E402

sbr.Engine.timing_enable = lambda self, on: None
sbr.Engine.timing_read = lambda self, stream=None: (1.0, 1.0, 1)
sys.argv = ["bench.py", "--warmup", "2", "--no-cpu-baseline"]
bench.main()
