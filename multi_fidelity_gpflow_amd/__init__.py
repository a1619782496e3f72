"""MI355X-native multi-fidelity GP engine (drop-in for qezlou/multi_fidelity_gpflow's hot path).

Public surface mirrors mfgpflow + the GPflow pieces it uses:
    SquaredExponential / RBF, LinearMultiFidelityKernel, MultiFidelityGPModel,
    LatentMFCoregionalizationSVGP, SingleBinSVGP, PowerSpecs, set_trainable, Parameter.
All arithmetic of the hot path runs in libmfgp.so (hand-written HIP for gfx950).
"""
from .params import Parameter, positive, set_trainable, parameter_dict, multiple_assign  # noqa: F401
from .kernels import (SquaredExponential, RBF, LinearMultiFidelityKernel,  # noqa: F401
                      LinearCoregionalization, SeparateIndependent)
from .models import MultiFidelityGPModel, Gaussian, CholeskyError, clear_session_pool  # noqa: F401
from .svgp import LatentMFCoregionalizationSVGP, SingleBinSVGP, initialize_W, initialize_W_pca  # noqa: F401
from .kernels import GraphMultiFidelityKernel  # noqa: F401
from .graph import GraphMultiFidelityGPModel  # noqa: F401
from .data import PowerSpecs, map_to_unit_cube, input_normalize  # noqa: F401
from . import data  # noqa: F401
from ._lib import MFGPError  # noqa: F401

__version__ = "0.1.0"
