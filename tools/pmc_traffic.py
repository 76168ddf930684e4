"""HBM bytes per launch of the bench's roofline kernels from two rocprofv3 --pmc passes.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json

FETCH_DIR / WRITE_DIR hold run_counter_collection.csv of `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
runs of `bench.py --no-graph` (separate passes: FETCH_SIZE takes 3 of the 4 TCC slots).
Corrections (MI355X_MICROARCH.md, HBM section): the counters are KiB; on gfx950 FETCH_SIZE
reports half the bytes of a 16-B-per-lane read (every read of these kernels is one), so it is
doubled; WRITE_SIZE is exact for 16-B stores.  Per kernel the median over the steady dispatches
is kept (the first dispatch of a run is a cold step).
"""
import csv
import json
import statistics
import sys

# probe name (bench.py) -> (kernel-name substring, grid size in threads or None, pick)
# pick "max": of several dispatches with the same name and grid per step, the ones whose FETCH
# is at least half the largest (MLP layer 1 forward shares its grid with MLP layer 2's dgrad)
KERNELS = {
    "fields_fwd": ("fields_fwd_kernel<128", None, None),
    # the claimed-row catch-up (fused with the row claims), the rolling window and the next-batch
    # prefetch's two passes (the bench's events bracket both; summed below)
    "adam_catchup": ("adam_claim2_conv_kernel<128", None, None),   # the step head (claims + bf16 images)
    "adam_window": ("adam_window2_kernel<128", None, None),
    "adam_prefetch": ("adam_prefetch2_kernel<128", None, None),
    "adam_pretag": ("adam_pretag_kernel", None, None),
    "gemm_mlp0": ("gemm_dma16_kernel<64, 128, false, false", "262144", "max"),
    "adam_touched": ("adam_touched_kernel<128", None, None),
    "adam_commit": ("adam_commit_kernel<128", None, None),
    "adam_tail": ("adam_tail_kernel<128", None, None),
    "wgrad_group": ("gemm_dma16_group_kernel<128, 128", None, None),
    "sum_jobs": ("sum_jobs_kernel", None, None),
}


def load(d, counter):
    import gzip
    import os
    rows = []
    path = f"{d}/run_counter_collection.csv"
    fh = open(path) if os.path.exists(path) else gzip.open(path + ".gz", "rt")   # gpu_pmc.sh gzips the passes
    for r in csv.DictReader(fh):
        if r["Counter_Name"] == counter:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], r["Grid_Size"], float(r["Counter_Value"])))
    return sorted(rows)


def select(rows, sub, grid):
    if grid in ("max", "min"):
        grids = [int(g) for _, name, g, _ in rows if sub in name]
        if not grids:
            return []
        grid = str(max(grids) if grid == "max" else min(grids))
    out = []
    for _, name, g, val in rows:
        if sub not in name:
            continue
        if grid is not None and (g == grid[1:] if grid.startswith("!") else g != grid):
            continue
        out.append(val)
    return out


def main():
    fdir, wdir, outp = sys.argv[1:4]
    fr, wr = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {}
    for key, (sub, grid, pick) in KERNELS.items():
        f, w = select(fr, sub, grid), select(wr, sub, grid)
        if not f or not w:
            continue
        if pick == "max":
            mf = max(f)
            idx = [i for i, v in enumerate(f) if v >= 0.5 * mf]
            f = [f[i] for i in idx]
            w = [w[i] for i in idx if i < len(w)]
        f, w = f[1:] or f, w[1:] or w                      # drop the cold first dispatch
        fb = 2.0 * statistics.median(f) * 1024.0
        wb = statistics.median(w) * 1024.0
        res[key] = {"kernel": sub, "fetch_bytes": round(fb), "write_bytes": round(wb),
                    "bytes_per_launch": round(fb + wb), "dispatches": len(f),
                    "note": "FETCH_SIZE KiB x 2 (gfx950 16-B-lane reads) + WRITE_SIZE KiB"}
    if "adam_prefetch" in res and "adam_pretag" in res:   # one fbn_adam_prefetch call = both passes
        for k in ("fetch_bytes", "write_bytes", "bytes_per_launch"):
            res["adam_prefetch"][k] += res["adam_pretag"][k]
        res["adam_prefetch"]["kernel"] += " + adam_pretag_kernel"
    json.dump(res, open(outp, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:14s} fetch {v['fetch_bytes'] / 1e6:9.2f} MB  write {v['write_bytes'] / 1e6:9.2f} MB  "
              f"total {v['bytes_per_launch'] / 1e6:9.2f} MB  (n={v['dispatches']})")


if __name__ == "__main__":
    main()
