"""enterprise_warp_amd — MI355X-native PTA log-likelihood behind enterprise_warp's surface.

Host side (Python): paramfile / noise-model JSON assembly (`warp`), the term
library (`models.StandardModels`), enterprise-style signals and parameters,
the `PTA` drop-in (`pta`), and the bilby adapters (`bilby_bridge`).
Device side: libewarp_hip.so (csrc/ewarp_hip.hip, gfx950 HIP kernels) behind
the C ABI in include/ewarp_hip.h.  See DESIGN.md.
"""
from . import constants, parameter, selections, signals  # noqa: F401
from .pulsar import Pulsar, load_bundle, save_bundle  # noqa: F401
from .pta import PTA, Engine  # noqa: F401
from .models import StandardModels  # noqa: F401
from .warp import Params, init_pta, parse_commandline, get_noise_dict  # noqa: F401
from .bilby_bridge import PTABilbyLikelihood, get_bilby_prior_dict  # noqa: F401

__version__ = "0.1.0"
