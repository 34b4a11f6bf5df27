"""Train step of the instant-ngp hot path (the reference Trainer.train_step
and train_one_epoch essentials, nerf/utils.py:453-609, 912-1072, with the
upstream cadence restored: density-grid update every 16 steps, §1.3.5).

MI355X specifics:
  * the whole forward + backward of a step (ray sampling, marching, grid
    encode, both MLPs, compositing, loss, backward) can be captured once into
    a hipGraph and replayed (`use_graph=True`), removing ~100 kernel-launch
    round trips of host overhead per step. This needs static shapes, i.e. a
    fixed `mean_count` (set from the measured sample count, exactly what
    update_extra_state does every 16 steps upstream);
  * the optimizer is torch's fused Adam (one kernel over every parameter),
    with GradScaler's unscale folded into it;
  * data parallel mode shards rays (each rank draws its own batch) and
    averages gradients with one RCCL all-reduce per parameter tensor.
"""
import torch
import torch.distributed as dist


def average_gradients(params, group=None):
    """Ray-sharded data parallelism: average every gradient over the ranks.
    One all-reduce per parameter tensor (hash table 12.2M fp32 + two MLPs):
    RCCL's AVG on GPU; SUM + scale elsewhere (gloo has no AVG)."""
    world = dist.get_world_size(group)
    if world == 1:
        return
    use_avg = dist.get_backend(group) == "nccl"
    for p in params:
        if p.grad is None:
            continue
        if use_avg:
            dist.all_reduce(p.grad, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=group)
            p.grad.div_(world)


class Trainer:
    def __init__(self, model, dataset, lr=1e-2, iters=30000, fp16=True, dt_gamma=0.0,
                 max_steps=1024, update_extra_interval=16, update_density=True,
                 distributed=False):
        self.model = model
        self.dataset = dataset
        self.fp16 = fp16
        self.dt_gamma = dt_gamma
        self.max_steps = max_steps
        self.update_extra_interval = update_extra_interval
        self.update_density = update_density
        self.distributed = distributed and dist.is_available() and dist.is_initialized()
        self.optimizer = torch.optim.Adam(model.get_params(lr), lr=lr, betas=(0.9, 0.99), eps=1e-15,
                                          fused=True)
        self.scheduler = torch.optim.lr_scheduler.LambdaLR(
            self.optimizer, lambda it: 0.1 ** min(it / iters, 1))
        self.scaler = torch.amp.GradScaler("cuda", enabled=fp16)
        self.global_step = 0
        self.graph = None
        self.static = None
        self.params = [p for g in self.optimizer.param_groups for p in g["params"]]

    # -------------------------------------------------------------- pieces
    def _forward_backward(self, data):
        images = data["images"]
        B, N, C = images.shape
        if C == 4:
            bg_color = torch.rand_like(images[..., :3])  # pixel-wise random background
            gt_rgb = images[..., :3] * images[..., 3:] + bg_color * (1 - images[..., 3:])
        else:
            bg_color = 1
            gt_rgb = images
        with torch.autocast("cuda", dtype=torch.float16, enabled=self.fp16,
                            cache_enabled=self.graph is None and self.static is None):
            outputs = self.model.render(data["rays_o"], data["rays_d"], staged=False,
                                        bg_color=bg_color, perturb=True, force_all_rays=False,
                                        dt_gamma=self.dt_gamma, max_steps=self.max_steps)
            pred_rgb = outputs["image"]
            loss = ((pred_rgb - gt_rgb) ** 2).mean(-1).mean()
        self.scaler.scale(loss).backward()
        return loss

    def _sync_grads(self):
        if self.distributed:
            average_gradients(self.params)

    def _optimizer_step(self):
        self._sync_grads()
        self.scaler.step(self.optimizer)
        self.scaler.update()
        self.scheduler.step()

    def _maybe_update_density(self):
        self.global_step += 1
        if self.update_density and self.global_step % self.update_extra_interval == 0:
            with torch.autocast("cuda", dtype=torch.float16, enabled=self.fp16):
                self.model.update_extra_state()

    # --------------------------------------------------------------- steps
    def train_step(self):
        """One eager step; returns the (device) loss tensor."""
        self.model.train()
        self.optimizer.zero_grad(set_to_none=True)
        data = self.dataset.sample()
        loss = self._forward_backward(data)
        self._optimizer_step()
        self._maybe_update_density()
        return loss.detach()

    def capture(self, warmup=3):
        """Capture forward+backward into a hipGraph (static mean_count)."""
        assert self.model.mean_count > 0, "capture needs a fixed mean_count (run eager steps first)"
        self.model.train()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.optimizer.zero_grad(set_to_none=True)
                self._forward_backward(self.dataset.sample())
                self._optimizer_step()
        torch.cuda.current_stream().wait_stream(side)
        self.optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        local_step = self.model.local_step
        with torch.cuda.graph(self.graph):
            self.static = self._forward_backward(self.dataset.sample())
        self.model.local_step = local_step

    def graph_step(self):
        """Replay the captured forward+backward, then the eager optimizer step."""
        self.graph.replay()
        self._optimizer_step()
        self.model.local_step += 1
        self._maybe_update_density()
        return self.static.detach()

    def step(self):
        return self.graph_step() if self.graph is not None else self.train_step()
