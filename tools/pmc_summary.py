"""Summarise rocprofv3 --pmc csv passes: per kernel (short name), mean counter value per dispatch.
FETCH_SIZE is reported x2 as well (gfx950 counts half the bytes of wide coalesced reads:
MI355X_MICROARCH.md, HBM section); sizes are in KB per the rocprofv3 derived counters.

With --json OUT, also writes the per-phase HBM traffic bench.py reports as roofline.traffic:
hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 of the phase's single kernel
(phases made of the shared radix-sort kernels are left out: their dispatches cannot be told
apart by name)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"lsr::(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


# bench phase -> the one kernel it launches (non-deterministic backward)
PHASE_KERNEL = {"preprocess": "k_preprocess", "emit": "k_emit", "tile_ranges": "k_tile_ranges",
                "render_fwd": "k_render_fwd_wave_mfma", "render_bwd": "k_render_bwd_wave",
                "preprocess_bwd": "k_preprocess_bwd", "preprocess_bwd_views": "k_preprocess_bwd_views"}

# the instantiations bench.py's timed step launches (C = 32, language operands split per batch)
BENCH_INSTANCE = {"render_fwd": ("k_render_fwd_wave_mfma<true>",),
                  "render_bwd": ("k_render_bwd_wave<true, true, false>", "k_render_bwd_wave<true, true>"),
                  "preprocess": ("k_preprocess<16, true>",)}


N_SIMD, N_XCD = 256 * 4, 8   # MI355X: 256 CUs x 4 SIMDs, 8 XCDs


def mfma_frac(c):
    """Matrix-core busy fraction of a dispatch: SQ_VALU_MFMA_BUSY_CYCLES (summed over the SIMDs;
    32 per v_mfma_f32_32x32x16_bf16, MI355X_MICROARCH.md) / (dispatch cycles x SIMDs), the dispatch
    cycles being GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs: checked against the kernel
    duration x 2.4 GHz)."""
    busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
    active = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"]) / N_XCD
    return busy / max(active * N_SIMD, 1.0)


STEP_FIRST, STEP_LAST = "k_preprocess<16, true>", "k_preprocess_bwd_views"


def step_bytes(d, counter):
    """Per bench step, the counter summed over EVERY dispatch of the step (the sorts, scans, fills
    and torch kernels included): a step runs from the batched preprocess (k_preprocess<16, true>)
    through the flush (k_preprocess_bwd_views); mean over the steps of the pass, in KB."""
    totals = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        rows = []
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    rows.append((int(row["Dispatch_Id"]), short(row.get("Kernel_Name", "")), float(row["Counter_Value"])))
        rows.sort()
        cur = None
        for _, k, v in rows:
            if k == STEP_FIRST:
                cur = 0.0
            if cur is not None:
                cur += v
                if k.split("<")[0] == STEP_LAST:
                    totals.append(cur)
                    cur = None
    return (sum(totals) / len(totals), len(totals)) if totals else (None, 0)


def main(d, json_out=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if not k.startswith("k_"):
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(acc):
        parts = []
        for c, v in sorted(acc[k].items()):
            mean = sum(v) / len(v)
            parts.append(f"{c}={mean:.4g}")
            if c == "FETCH_SIZE":
                parts.append(f"FETCH_SIZEx2_MB={2 * mean / 1024:.4g}")
            if c == "WRITE_SIZE":
                parts.append(f"WRITE_MB={mean / 1024:.4g}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in acc[k] and "GRBM_GUI_ACTIVE" in acc[k]:
            parts.append(f"MFMA_BUSY_FRAC={mfma_frac(acc[k]):.4g}")
        print(k, " ".join(parts))
    if json_out:
        import json
        res = {}
        for phase, kern in PHASE_KERNEL.items():
            ks = [k for k in acc if k.split("<")[0] == kern and "FETCH_SIZE" in acc[k] and "WRITE_SIZE" in acc[k]]
            if not ks:
                continue
            # several instantiations ran (the bench's batched path and its single-view leg): the
            # bench's own one, else the one dispatched most
            pref = [k for k in ks if k in BENCH_INSTANCE.get(phase, ())]
            ks = pref or sorted(ks, key=lambda k: -len(acc[k]["FETCH_SIZE"]))[:1]
            f = acc[ks[0]]
            fetch = sum(f["FETCH_SIZE"]) / len(f["FETCH_SIZE"])
            write = sum(f["WRITE_SIZE"]) / len(f["WRITE_SIZE"])
            res[phase] = dict(kernel=ks[0], fetch_size_kb=fetch, write_size_kb=write,
                              hbm_bytes_per_launch=int((2 * fetch + write) * 1024),
                              dispatches=len(f["FETCH_SIZE"]))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in f and "GRBM_GUI_ACTIVE" in f:
                res[phase]["mfma_busy_frac"] = round(mfma_frac(f), 4)
            if "SQ_INSTS_VALU" in f:   # wave-instructions per launch (each issues over 4 cycles on a SIMD)
                res[phase]["valu_insts_per_launch"] = int(sum(f["SQ_INSTS_VALU"]) / len(f["SQ_INSTS_VALU"]))
            if "SQ_ACTIVE_INST_VALU" in f and "SQ_WAVE_CYCLES" in f:
                # both count quad-cycles: the share of a resident wave's cycles that issue VALU
                res[phase]["valu_issue_per_wave"] = round(sum(f["SQ_ACTIVE_INST_VALU"]) / max(sum(f["SQ_WAVE_CYCLES"]), 1), 4)
        fetch, nf = step_bytes(d, "FETCH_SIZE")
        write, nw = step_bytes(d, "WRITE_SIZE")
        if fetch is not None and write is not None:
            res["_step"] = dict(fetch_size_kb=fetch, write_size_kb=write, steps=min(nf, nw),
                                hbm_bytes_per_step=int((2 * fetch + write) * 1024),
                                note="every dispatch from k_preprocess<16, true> through k_preprocess_bwd_views "
                                     "(sorts, scans, fills included), mean over the pass's steps")
            print(f"step: FETCH x2 {2 * fetch / 1024:.1f} MB + WRITE {write / 1024:.1f} MB = "
                  f"{(2 * fetch + write) / 1024:.1f} MB per step ({min(nf, nw)} steps)")
        res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, bench.py --steps 1 (8 views); "
                        "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md HBM section")
        with open(json_out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)
