from .ffmlp import FFMLP, ffmlp_forward, _ffmlp_forward

__all__ = ["FFMLP", "ffmlp_forward"]
