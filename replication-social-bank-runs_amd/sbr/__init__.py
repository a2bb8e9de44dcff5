"""sbr — MI355X batched equilibrium engine for "The Social Determinants of Bank
Runs" (drop-in for the β×u sweep hot path of Robin-Lenoir/replication-social-bank-runs).

The compute lives in libsbr.so (gfx950 HIP kernels behind the C ABI of
include/sbr.h); this package is the host-side mirror of the reference's
Julia call surface plus the multi-GPU sharding layer.
"""
from ._lib import STATUS, ArgumentError, SBRNativeError, header_symbols, load  # noqa: F401
from .engine import (  # noqa: F401
    Engine,
    LearningResults,
    LinearInterpolation,
    SolvedModel,
    default_engine,
    get_AW_functions,
    SolvedModelHetero,
    SolvedModelInterest,
    get_AW_functions_interest,
    solve_equilibrium_baseline,
    solve_equilibrium_hetero,
    solve_SInetwork_hetero,
    LearningResultsHetero,
    solve_equilibrium_interest,
    solve_equilibrium_social_learning,
    solve_learning,
)
from .grids import BaselineGrid, HeteroGrid, fig4_grid, fig5_grid, hetero_config4, hetero_script_grid, julia_range  # noqa: F401,E501
from .model import (  # noqa: F401
    EconomicParameters,
    LearningParameters,
    ModelParameters,
    ModelParametersHetero,
    LearningParametersHetero,
    EconomicParametersInterest,
    ModelParametersInterest,
)

__version__ = "0.1.0"
