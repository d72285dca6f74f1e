"""Device idle gaps inside one bench step from a rocprofv3 kernel trace (gpurun_out/prof):
the step spans from one batched preprocess launch to the next; prints every gap above a
threshold with the kernel that follows it, and the total.  Usage: trace_gaps.py [trace.csv] [us]"""
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/prof/**/*kernel_trace.csv", recursive=True)[0]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
starts = [i for i, x in enumerate(r) if "k_preprocess<" in x["Kernel_Name"] and "true>" in x["Kernel_Name"]]
if len(starts) < 3:
    starts = [i for i, x in enumerate(r) if "k_preprocess<" in x["Kernel_Name"]]
a, b = starts[-3], starts[-2]
busy_end, gaps, kern = None, 0.0, 0.0
for x in r[a:b]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    kern += (e - s) / 1e3
    if busy_end is not None and s > busy_end:
        g = (s - busy_end) / 1e3
        gaps += g
        if g > thr:
            print(f"gap {g:8.1f} us before {x['Kernel_Name'][:60]}")
    busy_end = e if busy_end is None else max(busy_end, e)
span = (int(r[b]["Start_Timestamp"]) - int(r[a]["Start_Timestamp"])) / 1e3
print(f"step span {span:.1f} us, kernels {kern:.1f} us, idle gaps {gaps:.1f} us ({100 * gaps / span:.1f} %)")
