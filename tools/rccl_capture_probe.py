"""Can RCCL collectives be captured in a hipGraph through torch.cuda.graph on
this image (one-rank `nccl` group on the box's GPU)? Captures
[scale -> reduce_scatter_tensor(AVG) -> all_gather_into_tensor (async, waited)]
and a variant with the reduce-scatter issued on a side stream that the
capture forks and joins, replays each, and checks the values.

    python tools/rccl_capture_probe.py
"""
import json
import os
import socket

import torch
import torch.distributed as dist


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {}
    n = 1 << 20
    x = (torch.arange(n, device=dev) % 97).half()
    shard = torch.empty(n, dtype=torch.float16, device=dev)
    full = torch.empty(n, dtype=torch.float16, device=dev)
    # eager first (communicator setup happens outside the capture)
    dist.reduce_scatter_tensor(shard, x, op=dist.ReduceOp.AVG)
    dist.all_gather_into_tensor(full, shard)
    torch.cuda.synchronize()
    for mode in ("same_stream", "side_stream"):
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            with torch.cuda.graph(g):
                x.mul_(2)
                if mode == "side_stream":
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        dist.reduce_scatter_tensor(shard, x, op=dist.ReduceOp.AVG)
                    torch.cuda.current_stream().wait_stream(side)
                else:
                    dist.reduce_scatter_tensor(shard, x, op=dist.ReduceOp.AVG)
                w = dist.all_gather_into_tensor(full, shard, async_op=True)
                w.wait()
                full.add_(1)
            ref = x.clone()
            for _ in range(3):
                g.replay()
                ref = ref * 2
            torch.cuda.synchronize()
            ok = torch.equal(full, ref + 1) and torch.equal(shard, ref)
            d = lambda a, b: float((a.float() - b.float()).abs().max())  # noqa: E731
            out[mode] = {"captured": True, "values_ok": bool(ok), "x_vs_ref": d(x, ref),
                         "shard_vs_ref": d(shard, ref), "full_vs_ref1": d(full, ref + 1),
                         "head": [x[:4].tolist(), shard[:4].tolist(), full[:4].tolist(), ref[:4].tolist()]}
        except Exception as e:  # noqa: BLE001
            out[mode] = {"captured": False, "error": repr(e)[:400]}
        x.copy_((torch.arange(n, device=dev) % 97).half())
        torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
