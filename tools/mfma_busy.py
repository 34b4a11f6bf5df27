"""MFMA-busy of the MLP kernels from tools/pmc_mlp.sh output: per kernel (name
prefix), SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) per
dispatch, averaged over dispatches, and the FLOP check
SQ_INSTS_VALU_MFMA_MOPS_F16 x 512.

    python tools/mfma_busy.py gpurun_out/<tag> [...]
"""
import collections
import csv
import glob
import sys


def main():
    for d in sys.argv[1:]:
        rows = collections.defaultdict(dict)  # (kernel, dispatch) -> counter -> value
        for f in glob.glob(d + "/*/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                key = next((k for k in ("k_nerf_bwd", "k_nerf_fwd", "k_density_fwd", "k_mlp_fwd", "k_mlp_bwd")
                            if k in name), None)
                if key is None:
                    continue
                rows[(key, f, r.get("Dispatch_Id", ""))][r["Counter_Name"]] = float(r["Counter_Value"])
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for (key, _, _), c in rows.items():
            for n, v in c.items():
                per[key][n].append(v)
        print(d)
        for key, c in sorted(per.items()):
            mean = {n: sum(v) / len(v) for n, v in c.items()}
            busy, gui = mean.get("SQ_VALU_MFMA_BUSY_CYCLES"), mean.get("GRBM_GUI_ACTIVE")
            frac = busy / (1024 * gui / 8) if busy is not None and gui else None
            mops = mean.get("SQ_INSTS_VALU_MFMA_MOPS_F16")
            print(f"  {key:18s} MFMA-busy {100 * frac:5.1f} %" if frac is not None else f"  {key:18s} (no busy pass)",
                  f"  FLOP/dispatch {mops * 512:.3e}" if mops else "", f"  dispatches {len(c.get('GRBM_GUI_ACTIVE', []))}")


if __name__ == "__main__":
    main()
