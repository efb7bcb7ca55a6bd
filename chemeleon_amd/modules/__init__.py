from chemeleon_amd.modules.chemeleon import Chemeleon

__all__ = ["Chemeleon"]
