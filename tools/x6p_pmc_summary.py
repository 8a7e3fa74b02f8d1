"""Per-kernel means of every counter in the passes tools/x6p_pmc.sh collected, plus
the trace's average duration and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / time)."""
import collections
import csv
import glob
import os
import sys


def short(name):
    if "X6pTile<" in name:
        return "x6p<" + name.split("X6pTile<", 1)[1].split(">")[0] + ">" + name.split(">", 2)[-1].split("(")[0][:8]
    for key in ("gemm_x6p_kernel", "gemm_nt_kernel", "split_w3_kernel"):
        if key in name:
            return key + name.split(key, 1)[1].split(")")[0][:90]
    return name.split("(")[0][:100]


def main():
    d = sys.argv[1]
    dur = collections.defaultdict(list)
    for p in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(set(dur) | set(cnt)):
        us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        row = {c: sum(v) / len(v) for c, v in cnt[k].items()}
        print("==", k, "n=%d" % len(dur[k]), "avg_us=%.2f" % us)
        if "GRBM_GUI_ACTIVE" in row and dur[k]:
            print("   clock_ghz=%.3f" % (row["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3)))
        wc = row.get("SQ_WAVE_CYCLES")
        for c in sorted(row):
            extra = ""
            if wc and c.startswith("SQ_") and c not in ("SQ_WAVE_CYCLES",) and "INSTS" not in c:
                extra = "  (/wave_cycles %.3f)" % (row[c] / wc)
            print("   %-28s %.4g%s" % (c, row[c], extra))


if __name__ == "__main__":
    main()
