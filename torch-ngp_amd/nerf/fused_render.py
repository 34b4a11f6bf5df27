"""Device-driven test render: the reference's inference loop (run_cuda with
training off, nerf/renderer.py:376-426) without its host round trip per
iteration.

The reference counts the alive rays on the host, picks
n_step = max(min(N // n_alive, 8), 1), runs march_rays -> network ->
composite_rays, compacts `rays_alive[rays_alive >= 0]` and loops until
step >= max_steps or no ray is alive: one device-to-host sync per iteration.
Here the loop state is a device record (csrc/raymarching.hip, RenderSlot)
that every kernel reads, the composite kernel appends the surviving rays to
the next iteration's list, and K iterations are captured in one hipGraph;
the host reads the state once per replay. Each iteration is 4 launches:

    render_march -> grid_encode (fused, world xyz, [L, M, 2])
    -> nerf_forward (sigma MLP + trunc_exp * density_scale + SH + colour MLP)
    -> render_composite (sigmoid of the colour logits, composite, survivors)

Per ray the arithmetic is the reference's under autocast (fp16 table and
MLPs, fp32 trunc_exp / SH / composite, half sigmoid), so images agree with
model.render(...) in eval mode (tests/test_gpu_render.py).
"""
import ctypes

import numpy as np
import torch

import _ngp_native as nat

_F32 = nat.DTYPE_CODE[torch.float32]


class FusedRenderer:
    def __init__(self, model, N, iters_per_graph=8, max_steps=1024, T_thresh=1e-4, dt_gamma=0.0):
        assert model.cuda_ray, "the renderer marches the density bitfield (cuda_ray=True)"
        enc, sn, cn = model.encoder, model.sigma_net, model.color_net
        assert enc.level_dim == 2 and enc.num_levels == 16 and enc.input_dim == 3
        assert (sn.hidden_dim == 64 and cn.hidden_dim == 64 and sn.input_dim == 32 and cn.input_dim == 32
                and 2 <= sn.num_layers <= 3 and 2 <= cn.num_layers <= 4), "ngp_nerf_forward shapes"
        assert iters_per_graph >= 2 and iters_per_graph % 2 == 0, "the state has two slots"
        self.model, self.N = model, int(N)
        self.K, self.max_steps, self.T_thresh, self.dt_gamma = int(iters_per_graph), int(max_steps), \
            float(T_thresh), float(dt_gamma)
        dev = model.density_bitfield.device
        self.dev = dev
        N = self.N

        def z(*shape, dtype=torch.float32):
            return torch.zeros(*shape, dtype=dtype, device=dev)

        h = torch.float16
        self.rays_o, self.rays_d = z(N, 3), z(N, 3)
        self.nears, self.fars, self.rays_t, self.noises = z(N), z(N), z(N), z(N)
        self.weights_sum, self.depth, self.image = z(N), z(N), z(N, 3)
        self.alive = [z(N, dtype=torch.int32), z(N, dtype=torch.int32)]
        # samples of one iteration: n_alive * n_step <= N
        self.xyzs, self.dirs, self.deltas = z(N, 3), z(N, 3), z(N, 2)
        self.enc_out, self.h_sigma, self.sigma = z(N, 32, dtype=h), z(N, 16, dtype=h), z(N)
        self.color_in, self.color_out = z(N, 32, dtype=h), z(N, 16, dtype=h)
        self.state = z(int(nat.lib().ngp_render_state_bytes()), dtype=torch.uint8)
        self.S = float(np.log2(enc.per_level_scale))
        self.w_half = [z(sn.weights.numel(), dtype=h), z(cn.weights.numel(), dtype=h)]
        nets = (sn, cn)
        self.mlp_img = [z(int(nat.lib().ngp_ffmlp_image_bytes(n.input_dim, n.hidden_dim, n.num_layers)),
                          dtype=torch.uint8) for n in nets]
        self._pk = dict(w=(ctypes.c_void_p * 2)(*[nat.ptr(t) for t in self.w_half]),
                        ins=(ctypes.c_uint32 * 2)(*[n.input_dim for n in nets]),
                        hid=(ctypes.c_uint32 * 2)(*[n.hidden_dim for n in nets]),
                        nl=(ctypes.c_uint32 * 2)(*[n.num_layers for n in nets]),
                        img=(ctypes.c_void_p * 2)(*[nat.ptr(t) for t in self.mlp_img]))
        self.graph = None
        self.iterations = 0  # device iterations of the last render (graph replays x K)

    def _stream(self):
        return nat.stream_of(self.rays_o)

    def load_weights(self):
        """fp16 copies of the MLP weights (autocast's casts) and their MFMA
        fragment images; the table is read in fp32 and rounded to half on load,
        the value autocast's cast gives. Call after the weights changed."""
        with torch.no_grad():
            self.w_half[0].copy_(self.model.sigma_net.weights.detach().reshape(-1))
            self.w_half[1].copy_(self.model.color_net.weights.detach().reshape(-1))
        pk = self._pk
        nat.check(nat.lib().ngp_ffmlp_pack(2, pk["w"], pk["ins"], pk["hid"], pk["nl"], pk["img"], self._stream()),
                  "ffmlp_pack")

    def _iteration(self, i):
        lib, P, s, m = nat.lib(), nat.ptr, self._stream(), self.model
        e, sn, cn, N = m.encoder, m.sigma_net, m.color_net, self.N
        cur, nxt = self.alive[i & 1], self.alive[(i + 1) & 1]
        cnt = lib.ngp_render_count(P(self.state), i)
        nat.check(lib.ngp_render_march(N, i, P(self.state), P(cur), P(self.rays_t), P(self.rays_o), P(self.rays_d),
                                       float(m.bound), self.dt_gamma, self.max_steps, m.cascade, m.grid_size,
                                       P(m.density_bitfield), P(self.fars), P(self.xyzs), P(self.dirs),
                                       P(self.deltas), P(self.noises), s), "render_march")
        nat.check(lib.ngp_grid_encode_forward_fused(P(self.xyzs), float(m.bound), P(e.embeddings), _F32,
                                                    P(e.offsets), P(self.enc_out), N, cnt, e.input_dim, e.level_dim,
                                                    e.num_levels, self.S, e.base_resolution, e.gridtype_id,
                                                    int(e.align_corners), e.interp_id, 0, s), "grid_encode_fused")
        nat.check(lib.ngp_nerf_forward(P(self.enc_out), P(self.mlp_img[0]), P(self.mlp_img[1]), N, cnt,
                                       sn.hidden_dim, sn.num_layers, cn.hidden_dim, cn.num_layers, P(self.h_sigma),
                                       P(self.sigma), P(self.color_in), P(self.dirs), float(m.density_scale),
                                       P(self.color_out), s), "nerf_forward")
        nat.check(lib.ngp_render_composite(N, i, self.max_steps, P(self.state), self.T_thresh, P(cur), P(nxt),
                                           P(self.rays_t), P(self.sigma), P(self.color_out), P(self.deltas),
                                           P(self.weights_sum), P(self.depth), P(self.image), s), "render_composite")

    def _iterations(self):
        for i in range(self.K):
            self._iteration(i)

    def _done(self):
        st = self.state[:16].view(torch.int32).cpu().numpy()  # slot 0 {count, n_alive, step, pad}
        return st[1] <= 0 or st[2] >= self.max_steps

    def capture(self):
        """One hipGraph of K loop iterations (the state makes spare iterations
        no-ops); render() replays it."""
        self.rays_o.zero_()
        self.rays_d[:, 2] = 1.0
        nat.check(nat.lib().ngp_render_init(self.N, nat.ptr(self.nears), nat.ptr(self.alive[0]),
                                            nat.ptr(self.rays_t), nat.ptr(self.weights_sum), nat.ptr(self.depth),
                                            nat.ptr(self.image), nat.ptr(self.state), self._stream()), "render_init")
        self._iterations()  # warm-up outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._iterations()
        self.graph = g

    @torch.no_grad()
    def render(self, rays_o, rays_d, bg_color=1, perturb=False):
        """rays_o / rays_d [N, 3] (or [1, N, 3]) -> dict(image [N, 3], depth
        [N], weights_sum [N]) as run_cuda's inference branch returns them:
        image + (1 - weights_sum) * bg_color, depth normalised to [near, far]."""
        m, lib, P, s = self.model, nat.lib(), nat.ptr, self._stream()
        self.rays_o.copy_(rays_o.reshape(self.N, 3))
        self.rays_d.copy_(rays_d.reshape(self.N, 3))
        aabb = m.aabb_train if m.training else m.aabb_infer
        nat.check(lib.ngp_near_far_from_aabb(P(self.rays_o), P(self.rays_d), P(aabb.contiguous()), self.N,
                                             float(m.min_near), P(self.nears), P(self.fars), s), "near_far")
        if perturb:
            self.noises.copy_(torch.rand(self.N, device=self.dev))
        else:
            self.noises.zero_()
        nat.check(lib.ngp_render_init(self.N, P(self.nears), P(self.alive[0]), P(self.rays_t),
                                      P(self.weights_sum), P(self.depth), P(self.image), P(self.state), s),
                  "render_init")
        replays = 0
        for _ in range(-(-self.max_steps // self.K)):  # each iteration advances step by >= 1
            if self.graph is not None:
                self.graph.replay()
            else:
                self._iterations()
            replays += 1
            if self._done():
                break
        self.iterations = replays * self.K
        ws = self.weights_sum
        image = self.image + (1 - ws).unsqueeze(-1) * bg_color
        depth = torch.clamp(self.depth - self.nears, min=0) / (self.fars - self.nears)
        return {"image": image, "depth": depth, "weights_sum": ws.clone()}
