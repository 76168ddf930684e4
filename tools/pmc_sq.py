"""Per-kernel PMC summary of rocprofv3 --pmc passes over bench.py (C3 step kernels).

  python tools/pmc_sq.py OUT.json PASS_DIR [PASS_DIR ...]

Each PASS_DIR holds run_counter_collection.csv (+ run_kernel_trace.csv) of one
`rocprofv3 --pmc <counters> --kernel-trace` run of `bench.py --no-graph` (tools/gpu_pmc.sh).
Kernels are grouped by (name, grid); per group the median over its steady dispatches (the first
is dropped) of every counter, and derived figures:

* cycles       = the kernel's duration (its --kernel-trace span) x F_CLK = 2.4 GHz, the MI355X peak
                 engine clock: a ratio over these cycles is a LOWER bound on the kernel's utilisation
                 (round 4 divided by GRBM_GUI_ACTIVE / 8, which counts the counter window around a
                 dispatch, not the dispatch: it derived 2.5-4.95 GHz clocks for kernels under ~30 us
                 and mis-scaled every ratio of theirs); grbm_clock_ghz keeps that derivation as a
                 diagnostic
* mfma_busy    = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs): fraction of the chip's matrix-
                 pipe cycles busy (a 32x32x16 bf16 MFMA keeps its SIMD busy 32 cycles);
                 mfma_tflops_at_busy = the bf16 rate those busy cycles imply at the kernel's clock
* valu_issue   = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (cycles x 1024): share of SIMD cycles
                 issuing VALU; valu_insts = SQ_INSTS_VALU per dispatch (wave instructions)
* hbm_bytes    = FETCH_SIZE x 2 (gfx950 16-B-lane reads are reported at half) + WRITE_SIZE, KiB
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

F_CLK_GHZ = 2.4       # MI355X peak engine clock (MI355X_MICROARCH.md)


def load_pass(d):
    trace = {}
    tp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            trace[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = defaultdict(dict)          # dispatch -> {counter: value}
    meta = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], int(r["Grid_Size"]))
    groups = defaultdict(list)
    for did in sorted(per):
        name, grid = meta[did]
        groups[(name.split("(")[0][:90], grid)].append((did, per[did], trace.get(did)))
    return groups


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    merged = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for key, disp in load_pass(d).items():
            steady = disp[1:] or disp
            for _, ctrs, us in steady:
                for c, v in ctrs.items():
                    merged[key][c].append(v)
                if us is not None:
                    merged[key]["duration_us"].append(us)
    res = []
    for (name, grid), ctrs in merged.items():
        m = {c: statistics.median(v) for c, v in ctrs.items()}
        d = {"kernel": name, "grid": grid, **{k: round(v, 3) for k, v in m.items()}}
        grbm = m.get("GRBM_GUI_ACTIVE", 0) / 8.0
        dur = m.get("duration_us", 0.0)
        cyc = dur * 1e3 * F_CLK_GHZ
        if grbm > 0 and cyc > 0:
            d["grbm_window_ratio"] = round(grbm / cyc, 3)
        if cyc > 0:
            d["cycles"] = round(cyc)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                d["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
                d["mfma_tflops_at_busy"] = round(d["mfma_busy"] * 1024 * 1024 * F_CLK_GHZ * 1e9 / 1e12, 1)
            if "SQ_ACTIVE_INST_VALU" in m:
                d["valu_issue"] = round(4 * m["SQ_ACTIVE_INST_VALU"] / (cyc * 1024), 4)
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            d["hbm_bytes"] = round(2 * m.get("FETCH_SIZE", 0) * 1024 + m.get("WRITE_SIZE", 0) * 1024)
        res.append(d)
    res.sort(key=lambda r: -r.get("duration_us", 0))
    json.dump(res, open(out, "w"), indent=1)
    for r in res[:30]:
        extra = "  ".join(f"{k} {r[k]}" for k in ("duration_us", "mfma_busy", "mfma_tflops_at_busy",
                                                 "valu_issue", "SQ_INSTS_VALU", "hbm_bytes") if k in r)
        print(f"{r['kernel'][:60]:60s} grid {r['grid']:8d}  {extra}")


if __name__ == "__main__":
    main()
