"""chemeleon_amd — MI355X-native (gfx950) implementation of Chemeleon's
reverse-diffusion sampling path, a drop-in for `chemeleon.Chemeleon` /
`chemeleon.modules.cspnet.CSPNet` on that path.

    from chemeleon_amd import Chemeleon
"""

from chemeleon_amd.modules.chemeleon import Chemeleon  # noqa: F401
from chemeleon_amd.modules.cspnet import CSPNet, DECODER_OUTPUTS  # noqa: F401

__all__ = ["Chemeleon", "CSPNet", "DECODER_OUTPUTS"]
__version__ = "0.1.0"
