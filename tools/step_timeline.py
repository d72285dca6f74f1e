"""One bench step's kernel timeline from a rocprofv3 kernel trace: every launch between two
consecutive batched preprocess launches with its start offset, duration and queue, plus per-kernel
totals.  Usage: step_timeline.py [trace.csv]"""
import collections
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/**/*kernel_trace.csv", recursive=True)[0]
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
starts = [i for i, x in enumerate(r) if "k_preprocess<" in x["Kernel_Name"] and "true>" in x["Kernel_Name"]]
a, b = starts[-3], starts[-2]
t0 = int(r[a]["Start_Timestamp"])
tot = collections.defaultdict(float)
cnt = collections.Counter()
qkey = "Queue_Id" if "Queue_Id" in r[a] else ("Stream_Id" if "Stream_Id" in r[a] else None)
for x in r[a:b]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    name = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("lsr::", "")[:48]
    tot[name] += (e - s) / 1e3
    cnt[name] += 1
    q = x.get(qkey, "") if qkey else ""
    print(f"{(s - t0) / 1e3:9.1f} +{(e - s) / 1e3:8.1f} us  q{q:>3}  {name}")
span = (int(r[b]["Start_Timestamp"]) - t0) / 1e3
print(f"\nstep span {span:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f} us  {cnt[k]:3d}x  {k}")
