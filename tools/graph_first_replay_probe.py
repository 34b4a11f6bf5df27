"""Is the first replay of a captured graph slow (upload on first launch)? The
Lego bench trainer: after capture + settle, the first-after-flush graph
(`_fresh`) is replayed for the first time, then again; a second trainer
uploads its graphs right after capture (hipGraphUpload) first.

    python tools/graph_first_replay_probe.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) * 1e3, 4)


def upload(g):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    return rc


def main():
    args = bench.parse()
    dev = torch.device("cuda:0")
    out = {}
    for mode in ("plain", "uploaded"):
        model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
        ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
        ft.step()
        ft.capture(warmup=2, multi=10)
        rc = None
        if mode == "uploaded":
            rc = [upload(g) for g in (ft.graph, ft.graph_multi, ft._fresh) if g is not None]
        r = {"upload_rc": rc}
        r["first_graph_replay_ms"] = timed(ft.step)
        r["second_graph_replay_ms"] = timed(ft.step)
        r["first_multi_replay_ms"] = timed(lambda: ft.graph_multi.replay())
        r["second_multi_replay_ms"] = timed(lambda: ft.graph_multi.replay())
        ft.flush()
        r["first_fresh_replay_ms"] = timed(ft.step)
        ft.step()
        ft.flush()
        r["second_fresh_replay_ms"] = timed(ft.step)
        r["eager_steps"] = ft.eager_steps
        out[mode] = r
        del ft, model
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
