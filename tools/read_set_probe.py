"""VERDICT r05 item 4 (exact deferred Adam): how much of the hash table one
training step READS. Deferred ("lazy") Adam could skip the sweep for a
4-value table group the step's forward does not read and whose gradient is
zero, and replay the skipped zero-gradient updates exactly before a later
forward reads it. That pays only if a large share of the groups Adam must
update (nonzero moments) goes unread per step.

After `steps` bench-configuration training steps (density updates on the
bench's cadence), one more step's marched samples (every sample, not only the
live rows) go through the reference-API grid forward + backward with a ones
gradient: the table entries with a nonzero gradient are exactly the entries
the forward gathered (a corner weight of exactly 0 aside). Per 4-value group
(the Adam sweep's unit) it reports: read this step, read in any of `window`
consecutive steps, nonzero moments, and nonzero moments AND unread (what a
deferred sweep would skip). Prints one JSON object.
    python tools/read_set_probe.py WORKLOAD [steps] [window]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def read_groups(ft, model):
    """Bool per 4-value group of the table: gathered by the last step's forward."""
    n = min(ft.sample_count(), ft.M)
    x = ft.xyzs[:n].clone()
    enc = model.encoder
    emb = enc.embeddings.detach().clone().requires_grad_(True)
    saved = enc.embeddings
    enc.embeddings = torch.nn.Parameter(emb)
    try:
        out = enc(x, bound=model.bound)
        out.float().sum().backward()
        g = enc.embeddings.grad.reshape(-1)
    finally:
        enc.embeddings = saved
    g4 = g[:g.numel() // 4 * 4].view(-1, 4)
    return (g4 != 0).any(1), n


def main():
    workload = sys.argv[1] if len(sys.argv) > 1 else "lego"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    window = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload(workload, dev, 1, args.num_rays)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    ft.capture(multi=args.graph_steps)
    done = 0
    while done < steps:
        k = min(64, steps - done)
        ft.run(k)
        done += k
        if done % 640 < 64:
            ft.update_density()
            ft.refresh_occupancy()
    per_step, union = [], None
    samples = []
    for _ in range(window):
        ft.step()
        torch.cuda.synchronize()
        r, n = read_groups(ft, model)
        samples.append(n)
        per_step.append(float(r.float().mean()))
        union = r if union is None else (union | r)
    ft.flush()
    n4 = union.numel()
    m = ft.exp_avg[:4 * n4].view(-1, 4)
    v = ft.exp_avg_sq[:4 * n4].view(-1, 4)
    active = ((m != 0) | (v != 0)).any(1)
    offs = model.encoder.offsets.cpu().tolist()
    levels = []
    for lv in range(len(offs) - 1):
        a, b = offs[lv] * 2 // 4, offs[lv + 1] * 2 // 4  # entries x 2 channels / 4 values per group
        levels.append({"level": lv, "groups": b - a, "read_last_step": round(float(r[a:b].float().mean()), 4),
                       "active": round(float(active[a:b].float().mean()), 4)})
    out = {"workload": workload, "steps": steps, "samples_per_step": samples,
           "table_groups": int(n4),
           "read_per_step_frac": [round(f, 4) for f in per_step],
           "read_in_window_frac": round(float(union.float().mean()), 4), "window": window,
           "active_frac": round(float(active.float().mean()), 4),
           "active_unread_last_step_frac": round(float((active & ~r).float().mean()), 4),
           "per_level": levels}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
