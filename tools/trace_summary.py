"""Per-kernel duration summary of rocprofv3 --kernel-trace CSV directories.

  python tools/trace_summary.py gpurun_out/pv_main [gpurun_out/pv_dbg1 ...]

One table per directory: dispatches, mean and median microseconds per (kernel, grid,
workgroup), sorted by total time; then the summed median time of one single-query
forward's kernel classes when the trace is a tools/latency.py --encoder-seq-lens run.
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    path = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not path:
        return None
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (name[:70], r.get("Grid_Size_X", ""), r.get("Workgroup_Size_X", ""))
        out[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


def main():
    for d in sys.argv[1:]:
        t = load(d)
        print("==", d)
        if t is None:
            print("   (no trace)")
            continue
        for k, v in sorted(t.items(), key=lambda kv: -sum(kv[1])):
            v = sorted(v)
            print("%6d  mean %7.2f  med %7.2f us  %s grid %s wg %s" % (len(v), sum(v) / len(v), v[len(v) // 2], *k))


if __name__ == "__main__":
    main()
