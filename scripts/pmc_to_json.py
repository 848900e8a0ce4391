"""Per-launch HBM traffic from a PMC summary (scripts/pmc_summary.py output)
-> profiles/pmc_latest.json, read by bench.py for roofline.traffic.

MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KB) = TCC_EA0_RDREQ x 64 B and
on gfx950 reports half of the bytes of wide reads -> read bytes = 2 x
FETCH_SIZE x 1024; WRITE_SIZE (KB) is exact for wide stores and atomics.
Infinity-Cache hits are included (fabric-side counters)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

summary, out, config, semantics = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
d = json.load(open(summary))
res = {}
for name, c in d.items():
    key = name.split("(")[0].split("<")[0].strip()
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res[key] = 2.0 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
h = hashlib.sha256(open(os.path.join(ROOT, "vq-gnn_amd", "lib", "libvqgnn.so"), "rb").read())
json.dump({"config": config, "semantics": semantics, "hbm_bytes_per_launch": res,
           "lib_sha256": h.hexdigest(), "git_head": os.environ.get("GIT_HEAD"),
           "rule": "2*FETCH_SIZE + WRITE_SIZE (KB->B), per launch, gfx950 wide-read correction",
           "source": summary}, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
