"""enterprise_extensions.model_utils surface used by the reference's driver
(examples/run_example_paramfile.py:10, :25-45): `setup_sampler`,
`HyperModel`, `get_parameter_groups`.  With this module the driver's PTMCMC
branch runs with only its imports changed
(`from enterprise_warp_amd import model_utils`)."""
from .hypermodel import HyperModel  # noqa: F401
from .ptmcmc import JumpProposal, PTSampler, get_parameter_groups, setup_sampler  # noqa: F401
