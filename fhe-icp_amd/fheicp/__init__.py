"""fheicp — MI355X-native encrypted-similarity engine (gfx950 HIP kernels).

Drop-in replacement for the Concrete-ML estimator behind
shipstone-labs/fhe-icp's encrypted pairwise compare (fhe_similarity.py:88-167,
batch_operations.py:206-284). See DESIGN.md and INTEGRATION.md.
"""
from .params import SchemeParams, TOY, noise_report, params_for_bits  # noqa: F401
from ._lib import FheError, LIB_PATH  # noqa: F401

__all__ = ["SchemeParams", "TOY", "noise_report", "params_for_bits", "FheError", "LIB_PATH"]
