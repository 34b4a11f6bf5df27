"""CPU: the C-ABI boundary and the host-side mirror of the reference interface.

No kernel is launched here (no GPU in the build container): the library must
load and export every symbol include/ngp_hip.h declares, the ctypes table
must match the header, argument checks must raise the reference's errors,
and the product code must never import the oracle.
"""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ngp_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ngp_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ["ngp_grid_encode_forward", "ngp_grid_encode_backward", "ngp_grad_total_variation",
                 "ngp_near_far_from_aabb", "ngp_sph_from_ray", "ngp_morton3D", "ngp_morton3D_invert",
                 "ngp_packbits", "ngp_march_rays_train", "ngp_composite_rays_train_forward",
                 "ngp_composite_rays_train_backward", "ngp_march_rays", "ngp_composite_rays",
                 "ngp_sh_encode_forward", "ngp_sh_encode_backward", "ngp_ffmlp_forward",
                 "ngp_ffmlp_inference", "ngp_ffmlp_backward", "ngp_ffmlp_allocate_splitk",
                 "ngp_ffmlp_free_splitk", "ngp_adam_step"]:
        assert name in fns, name


def test_library_exports_every_header_symbol():
    import _ngp_native as nat
    if not os.path.exists(nat.LIB_PATH):
        pytest.skip("libngp_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(nat.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), f"{name} declared in ngp_hip.h but not exported"


def test_ctypes_table_matches_header():
    import _ngp_native as nat
    assert sorted(nat.SIGNATURES) == header_functions()
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name, argtypes in nat.SIGNATURES.items():
        m = re.search(name + r"\s*\(([^)]*)\)", src)
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(argtypes), name


def test_abi_version_and_error_channel():
    import _ngp_native as nat
    if not os.path.exists(nat.LIB_PATH):
        pytest.skip("libngp_hip.so not built")
    assert nat.lib().ngp_abi_version() == 1
    assert isinstance(nat.lib().ngp_last_error(), bytes)
    # argument validation happens before any device work -> usable without a GPU
    rc = nat.lib().ngp_sh_encode_forward(None, None, 4, 2, 4, None, 0, None)
    assert rc == -1 and b"input dim" in nat.lib().ngp_last_error()
    rc = nat.lib().ngp_ffmlp_forward(None, None, 16, 32, 16, 256, 2, 0, 6, None, None, None)
    assert rc == -3 and b"hidden_dim" in nat.lib().ngp_last_error()
    rc = nat.lib().ngp_grid_encode_forward(None, None, None, None, 4, 3, 2, 65, 1.0, 16, None, 0, 0, 0,
                                           0, 0, None)
    assert rc == -1


def test_backend_rejects_cpu_tensors_like_torch_check():
    from gridencoder.backend import _backend as gb
    from raymarching.backend import _backend as rb
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        gb.grid_encode_forward(x, torch.zeros(8, 2), torch.zeros(2, dtype=torch.int32),
                               torch.zeros(1, 4, 2), 4, 3, 2, 1, 1.0, 16, None, 0, False, 0)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        rb.near_far_from_aabb(x, x, torch.zeros(6), 4, 0.2, torch.zeros(4), torch.zeros(4))


def test_operator_surface_names_match_reference():
    """The reference's pybind11 names (gridencoder/src/bindings.cpp:5-9,
    raymarching/src/bindings.cpp:5-18, shencoder/src/bindings.cpp:5-8,
    ffmlp/src/bindings.cpp:5-11) all exist on the _backend shims, and the
    wrapper modules export the reference's autograd ops."""
    from ffmlp.backend import _backend as fb
    from gridencoder.backend import _backend as gb
    from raymarching.backend import _backend as rb
    from shencoder.backend import _backend as sb
    for ns, names in ((gb, ["grid_encode_forward", "grid_encode_backward", "grad_total_variation"]),
                      (rb, ["near_far_from_aabb", "sph_from_ray", "morton3D", "morton3D_invert",
                            "packbits", "march_rays_train", "composite_rays_train_forward",
                            "composite_rays_train_backward", "march_rays", "composite_rays"]),
                      (sb, ["sh_encode_forward", "sh_encode_backward"]),
                      (fb, ["ffmlp_forward", "ffmlp_inference", "ffmlp_backward", "allocate_splitk",
                            "free_splitk"])):
        for n in names:
            assert callable(getattr(ns, n)), n
    import raymarching
    for n in ["near_far_from_aabb", "sph_from_ray", "morton3D", "morton3D_invert", "packbits",
              "march_rays_train", "composite_rays_train", "march_rays", "composite_rays"]:
        assert callable(getattr(raymarching, n))
    from ffmlp import FFMLP
    from gridencoder import GridEncoder
    from shencoder import SHEncoder
    assert GridEncoder and SHEncoder and FFMLP


def test_modules_construct_on_cpu_with_reference_shapes():
    import _ngp_native as nat
    if not os.path.exists(nat.LIB_PATH):
        pytest.skip("libngp_hip.so not built")
    from encoding import get_encoder
    from nerf.network_ff import NeRFNetwork
    net = NeRFNetwork(bound=1, cuda_ray=True)
    assert net.encoder.embeddings.numel() == 12239728
    assert net.sigma_net.weights.numel() == 64 * (32 + 64 + 16) == 7168
    assert net.color_net.weights.numel() == 64 * (32 + 128 + 16) == 11264
    assert net.density_bitfield.numel() == 128 ** 3 // 8 and net.cascade == 1
    assert NeRFNetwork(bound=2, cuda_ray=True).cascade == 2
    enc, d = get_encoder("sphere_harmonics")
    assert d == 16
    enc, d = get_encoder("frequency", multires=6)
    assert d == 3 + 3 * 6 * 2
    # FFMLP init is the reference's: manual_seed(42), U(+-sqrt(3/hidden))
    from ffmlp import FFMLP
    a = FFMLP(32, 16, 64, 2).weights.detach().clone()
    torch.manual_seed(42)
    b = torch.zeros(7168).uniform_(-(3 / 64) ** 0.5, (3 / 64) ** 0.5)
    assert torch.equal(a, b)


def test_product_code_never_imports_oracle():
    pkg = os.path.join(ROOT, "torch-ngp_amd")
    offenders = []
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                if re.search(r"^\s*(import|from)\s+oracle\b", src, flags=re.M) or "ngp_oracle" in src:
                    offenders.append(f)
    assert not offenders, offenders
