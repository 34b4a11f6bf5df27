from .sphere_harmonics import SHEncoder, sh_encode, _sh_encoder

__all__ = ["SHEncoder", "sh_encode"]
