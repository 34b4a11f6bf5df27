from .freq import FreqEncoder, freq_encode, _freq_encoder

__all__ = ["FreqEncoder", "freq_encode"]
