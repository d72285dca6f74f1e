import csv, glob, re, sys, collections
path = glob.glob("gpurun_out/tprof/**/*kernel_trace.csv", recursive=True)[0]
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
n = len(r)
r = r[n // 2:]   # second half: steady state
t0, t1 = int(r[0]["Start_Timestamp"]), max(int(x["End_Timestamp"]) for x in r)
busy_end, gaps, kern = None, 0.0, collections.Counter()
for x in r:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    kern[re.sub(r"\(.*", "", x["Kernel_Name"]).replace("void ", "")[:50]] += (e - s) / 1e3
    if busy_end is not None and s > busy_end:
        gaps += (s - busy_end) / 1e3
    busy_end = e if busy_end is None else max(busy_end, e)
span = (t1 - t0) / 1e3
print(f"span {span:.0f} us, idle {gaps:.0f} us ({100*gaps/span:.1f} %), kernels {sum(kern.values()):.0f} us, launches {len(r)}")
for k, v in kern.most_common(25):
    print(f"{v:10.0f} us {k}")
