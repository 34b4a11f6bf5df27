from .grid import GridEncoder, grid_encode, _grid_encode

__all__ = ["GridEncoder", "grid_encode"]
