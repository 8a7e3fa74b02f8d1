"""Summarise one round of profiles/run_profiles.sh output into profiles/<round>/.

  python3 tools/summarize_profiles.py gpurun_out/prof_r1 profiles/r1

Writes
  kernel_stats.csv     rocprofv3 --stats summary of the traced bench run (copied)
  trace_bench.json     the bench JSON line of the traced run
  pmc_fetch_write.csv  per kernel: dispatches, FETCH_SIZE / WRITE_SIZE (KB, averaged per
                       dispatch) and HBM bytes per dispatch = 2*FETCH + WRITE (gfx950
                       FETCH_SIZE counts half of a wide streaming read, MI355X_MICROARCH.md)
  pmc_sq.csv           per kernel: effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration),
                       MFMA busy fraction of all SIMD cycles, wait / issue-stall / active
                       shares of wave cycles, LDS bank-conflict cycles
and refreshes profiles/pmc_traffic.json (the source of bench.py's roofline `traffic`).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

CUS = 256


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].strip()


def find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    return hits[0] if hits else None


def counters(d):
    """({kernel: {counter: [value per dispatch]}}, {kernel: [duration ns per dispatch]})"""
    path = find(d, "counter_collection.csv")
    out = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    if not path:
        return out, dur
    seen = set()
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (r.get("Dispatch_Id"), k)
            if key not in seen and r.get("End_Timestamp"):
                seen.add(key)
                dur[k].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out, dur


def dispatches(d, counter):
    """[(dispatch id, kernel, grid size, value of `counter`)] in dispatch order."""
    path = find(d, "counter_collection.csv")
    rows = []
    if not path:
        return rows
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
            rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), grid, float(r["Counter_Value"])))
    rows.sort()
    return rows


def classify(rows):
    """Dispatch -> bench.py kernel class, or None.  The encoder GEMM classes are the
    headline shape's launches only: a class's most common grid (the full-M launches of
    the L = 32 batch; the CLS-only last layer and other shapes drop out), and the shared
    residual-epilogue instantiation is split by what precedes it (attention -> out-proj,
    FFN-up -> FFN-down)."""
    out = []
    prev = ""
    for did, k, grid, v in rows:
        cls = None
        mx = re.search(X6P_GEMM, k)
        if mx:  # the split-f32 encoder GEMMs on pre-split weights (K2p)
            e = mx.group(1)
            cls = {"0": "qkv_gemm_x6p", "1": "ffn_up_gemm_x6p", "2": "ffn_up_gemm_x6p"}.get(e)
            if e == "3":
                cls = "out_proj_gemm_x6p" if "attention" in prev else \
                    "ffn_down_gemm_x6p" if ("gemm_x6p_kernel" in prev or "gemm_nt_kernel" in prev) else None
        elif re.search(EXACT_GEMM + r"0" + LN_ARG, k):
            cls = "qkv_gemm"
        elif re.search(EXACT_GEMM + r"[12]" + LN_ARG, k):
            cls = "ffn_up_gemm"
        elif re.search(EXACT_GEMM + r"3" + LN_ARG, k):
            cls = "out_proj_gemm" if "attention" in prev else "ffn_down_gemm" if "gemm_nt_kernel" in prev else None
        else:
            for c, pat in CLASSES.items():
                if c not in ("qkv_gemm", "ffn_up_gemm", "out_proj_gemm", "ffn_down_gemm") and re.search(pat, k):
                    cls = c
        out.append((cls, grid, v))
        prev = k
    by = defaultdict(lambda: defaultdict(list))
    for cls, grid, v in out:
        if cls:
            by[cls][grid].append(v)
    res = {}
    for cls, grids in by.items():
        grid, vals = max(grids.items(), key=lambda kv: len(kv[1]))
        vals = sorted(vals)
        res[cls] = (vals[len(vals) // 2], len(vals), grid)
    return res


def mean(v):
    return sum(v) / len(v) if v else 0.0


# the exact-f32 encoder GEMM (X6 = false, BF16 = false, optional slice-depth parameter)
# followed by its epilogue id
EXACT_GEMM = r"gemm_nt_kernel<mq::F32Tile<\d+, \d+, \d+, \d+, false, \d+, false(, \d+)?(, (true|false))?>, "
# the split-f32 GEMM on pre-split weights (gemm_x6p.hip), its epilogue id captured
X6P_GEMM = r"gemm_x6p_kernel<mq::X6pTile<[^>]*>, (\d)>"
# ... then gemm_nt_kernel's LN_IN argument (r4: LayerNorm on load, false by default)
LN_ARG = r"(, (true|false))?>"
# bench.py kernel class -> kernel-name regex (the encoder GEMM classes are resolved per
# dispatch by classify())
CLASSES = {
    "flat_search_kernel": r"flat_search_kernel<mq::F32Tile<2, 2, 2, 2, false, \d, false(, \d+)?>, \d+>",
    "flat_search_kernel_x6": r"flat_search_kernel<mq::F32Tile<2, 2, 2, 2, true, \d, false(, \d+)?>, 8>",
    "flat_search_kernel_bf16": r"flat_search_kernel<mq::F32Tile<2, 2, 2, 2, false, \d, true(, \d+)?>, 8>",
    "bf16_thresh_kernel": r"bf16_thresh_kernel<\d+, 1(, false)?>",  # (unmasked)
    "bf16_thresh_sample": r"bf16_thresh_kernel<\d+, 0(, false)?>",
    "i8_thresh_kernel": r"i8_thresh_kernel<\d, 1, 1>",
    "i8_thresh_sample": r"i8_thresh_kernel<\d, 1, 0>",
    "qkv_gemm": r"gemm_nt_kernel<mq::F32Tile<\d, \d, \d, \d, false, \d, false>, 0>",
    "ffn_up_gemm": r"gemm_nt_kernel<mq::F32Tile<\d, \d, \d, \d, false, \d, false>, [12]>",
    "out_proj_gemm": r"gemm_nt_kernel<mq::F32Tile<\d, \d, \d, \d, false, \d, false>, 3>",
    "ffn_down_gemm": r"gemm_nt_kernel<mq::F32Tile<\d, \d, \d, \d, false, \d, false>, 3>",
}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = find(os.path.join(src, "trace"), "kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    tb = os.path.join(src, "trace_bench.json")
    if os.path.exists(tb):
        shutil.copy(tb, os.path.join(dst, "trace_bench.json"))

    fetch, _ = counters(os.path.join(src, "fetch"))
    write, _ = counters(os.path.join(src, "write"))
    rows = []
    for k in sorted(set(fetch) | set(write)):
        fv = fetch[k].get("FETCH_SIZE", [])
        wv = write[k].get("WRITE_SIZE", [])
        f_kb, w_kb = mean(fv), mean(wv)
        rows.append([k, len(fv) or len(wv), round(f_kb, 1), round(w_kb, 1),
                     int(2 * f_kb * 1024 + w_kb * 1024)])
    if rows:
        with open(os.path.join(dst, "pmc_fetch_write.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatches", "FETCH_SIZE_KB_avg", "WRITE_SIZE_KB_avg",
                        "hbm_bytes_corrected"])
            w.writerows(rows)

    sq, dur = counters(os.path.join(src, "sq"))
    srows = []
    for k in sorted(sq):
        c = {n: mean(v) for n, v in sq[k].items()}
        ns = mean(dur.get(k, []))
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES over every
        # SIMD: the chip's SIMD-cycles in the dispatch = gui / 8 * 4 SIMDs * CUs
        simd_cycles = gui / 8 * 4 * CUS
        srows.append([
            k, len(sq[k].get("SQ_WAVE_CYCLES", [])), round(ns / 1e3, 2),
            round(gui / 8 / ns, 3) if ns else "",
            round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles, 4) if simd_cycles else "",
            round(c.get("SQ_WAIT_ANY", 0.0) / wave, 4) if wave else "",
            round(c.get("SQ_WAIT_INST_ANY", 0.0) / wave, 4) if wave else "",
            round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wave, 4) if wave else "",
            int(c.get("SQ_LDS_BANK_CONFLICT", 0.0)),
        ])
    if srows:
        with open(os.path.join(dst, "pmc_sq.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatches", "avg_us_profiled", "eff_clock_ghz", "mfma_busy",
                        "wait_any_share", "issue_stall_share", "active_share",
                        "lds_bank_conflict_cycles"])
            w.writerows(srows)

    fcls = classify(dispatches(os.path.join(src, "fetch"), "FETCH_SIZE"))
    wcls = classify(dispatches(os.path.join(src, "write"), "WRITE_SIZE"))
    if fcls:
        traffic = {"note": "HBM bytes per launch = 2*FETCH_SIZE(KB)*1024 + WRITE_SIZE(KB)*1024 "
                           "(gfx950 FETCH_SIZE halves wide streaming reads, MI355X_MICROARCH.md "
                           "HBM section), the median over the class's launches of the headline "
                           "shape (its most common grid; out-proj / FFN-down told apart by the "
                           "preceding launch); rocprofv3 --pmc passes of profiles/run_profiles.sh, "
                           "summarised by tools/summarize_profiles.py",
                   "source": dst, "launches": {}}
        for cls, (fkb, n, grid) in sorted(fcls.items()):
            wkb = wcls.get(cls, (0.0, 0, ""))[0]
            traffic[cls] = int(2 * fkb * 1024 + wkb * 1024)
            traffic["launches"][cls] = {"dispatches": n, "grid": grid, "fetch_kb": round(fkb, 1),
                                        "write_kb": round(wkb, 1)}
        with open(os.path.join(dst, "pmc_traffic_classes.json"), "w") as f:
            json.dump(traffic, f, indent=1)
        with open(os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
