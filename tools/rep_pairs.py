"""Cold vs warm duration of each few-row launch from a kernel trace of a -DMQ_ROWS_REPEAT
measurement build (every launch runs twice back to back: dispatch 2j of a kernel is the
cold run, 2j+1 the same launch with its weights already pulled into L2 / MALL).

  python tools/rep_pairs.py gpurun_out/rowsrep_trace
"""
import collections
import csv
import glob
import os
import sys


def main():
    path = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "rows" not in name:
            continue
        key = (name[:60], r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
        seq[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot_c = tot_w = 0.0
    for k, v in sorted(seq.items(), key=lambda kv: -sum(kv[1])):
        cold, warm = sorted(v[0::2]), sorted(v[1::2])
        if not warm:
            continue
        mc, mw = cold[len(cold) // 2], warm[len(warm) // 2]
        tot_c += mc * len(cold)
        tot_w += mw * len(warm)
        print("%5d pairs  cold med %6.2f us  warm med %6.2f us  %s" % (len(warm), mc, mw, k))
    print("sum of medians x count: cold %.1f us  warm %.1f us" % (tot_c, tot_w))


if __name__ == "__main__":
    main()
