"""CPU: the Config 1 pure-PyTorch path (oracle/torch_nerf.py) that bench.py
times as the CPU baseline: its hash grid / SH / near-far restatements against
the C oracle, and a train step that runs and learns."""
import numpy as np
import torch

import oracle
from oracle import torch_nerf as tn


def test_torch_hashgrid_matches_oracle():
    torch.manual_seed(0)
    enc = tn.TorchHashGrid(log2_hashmap_size=14)
    with torch.no_grad():
        enc.embeddings.normal_(0, 0.1)
    x = torch.rand(500, 3) * 2 - 1
    got = enc(x).detach().numpy()
    x01 = ((x + 1) / 2).numpy().astype(np.float32)
    ref, _ = oracle.grid_encode_forward(x01, enc.embeddings.detach().numpy(), np.array(enc.offsets, np.int32),
                                        enc.per_level_scale, 16)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    assert np.array_equal(np.array(enc.offsets, np.int32), oracle.grid_offsets(3, 16, 2, 16, enc.per_level_scale, 14))


def test_sh_and_near_far_match_oracle():
    rng = np.random.default_rng(1)
    d = rng.standard_normal((300, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    np.testing.assert_allclose(tn.sh_encode4(torch.from_numpy(d)).numpy(), oracle.sh_encode(d, 4), atol=2e-6)
    o = (rng.standard_normal((300, 3)) * 2).astype(np.float32)
    aabb = np.array([-1, -1, -1, 1, 1, 1], np.float32)
    n, f = tn.near_far_from_aabb(torch.from_numpy(o), torch.from_numpy(d), torch.from_numpy(aabb))
    rn, rf = oracle.near_far_from_aabb(o, d, aabb, 0.2)
    hit = rn < 1e30
    assert np.array_equal(hit, n.numpy() < 1e30)
    np.testing.assert_allclose(n.numpy()[hit], rn[hit], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(f.numpy()[hit], rf[hit], rtol=1e-5, atol=1e-6)


def test_config1_train_step_learns():
    torch.manual_seed(0)
    model = tn.TorchNeRF(num_steps=64)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-15)
    batches = tn.lego_batches(1, num_rays=256)
    losses = [tn.train_step(model, opt, *batches[0]) for _ in range(15)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
    assert model.encoder.embeddings.grad is not None and model.encoder.embeddings.grad.abs().sum() > 0
