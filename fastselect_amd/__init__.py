"""fastselect_amd -- MI355X-native Relief-family feature scoring.

Drop-in for the Relief path of ``fast_select`` (GavinLynch04/FastSelect):
``ReliefF``, ``SURF`` (``use_star=True``: SURF*), ``MultiSURF``
(``use_star=True``: MultiSURF*; also as ``SURFstar`` / ``MultiSURFstar``, the
scikit-rebate names) and the ``TuRF`` meta-estimator, with the same
scikit-learn surface.  Scoring runs in hand-written HIP kernels for gfx950
(``fastselect_amd/csrc``) behind the C ABI in ``include/fastselect_amd.h``;
``fastselect_amd.parallel`` shards MultiSURF over one process per GPU.

Importing the package loads the native library; it fails loudly if the
library has not been built.
"""
from . import _lib
from .MultiSURF import MultiSURF
from .ReliefF import ReliefF
from .SURF import SURF
from .star import MultiSURFstar, SURFstar
from .TuRF import TuRF

__version__ = "0.1.0"
__all__ = ["ReliefF", "SURF", "MultiSURF", "SURFstar", "MultiSURFstar", "TuRF"]


def gpu_available() -> bool:
    """True when at least one HIP device is visible to the native library."""
    return _lib.gpu_available()
