"""Summarise rocprofv3 PMC passes: per kernel, mean counter value per dispatch."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/p*/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for k, cs in acc.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    if dur.get(k):
        d["dur_ns_mean"] = sum(dur[k]) / len(dur[k])
    out[k] = d
for k, d in sorted(out.items(), key=lambda kv: -kv[1].get("dur_ns_mean", 0)):
    print(k[:60])
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {v:16.1f}")
json.dump(out, open(f"{root}/summary.json", "w"), indent=1)
