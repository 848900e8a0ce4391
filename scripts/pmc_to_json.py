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
res, counters = {}, {}
for name, c in d.items():
    key = name.split("(")[0].split("<")[0].strip()
    # kernels of one name (template instances: the warm-up feature_update's
    # W = 4 assign beside the step's W = 8) keep the longest-running instance
    if key in counters and c.get("dur_ns_mean", 0) <= counters[key].get("dur_ns_mean", 0):
        continue
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res[key] = 2.0 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
    # the SQ counters bench.py prices the assign with (MFMA and VALU issue,
    # wait fraction), per launch
    counters[key] = {k: v for k, v in c.items()
                     if k.startswith("SQ_") or k in ("GRBM_GUI_ACTIVE", "dur_ns_mean")}


def git_head():
    """The commit the counters belong to: $GIT_HEAD (the GPU box gets no .git
    directory), else the local repository's HEAD, else null."""
    if os.environ.get("GIT_HEAD"):
        return os.environ["GIT_HEAD"]
    try:
        import subprocess
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True,
                              text=True, check=True).stdout.strip() or None
    except Exception:
        return None


h = hashlib.sha256(open(os.path.join(ROOT, "vq-gnn_amd", "lib", "libvqgnn.so"), "rb").read())
json.dump({"config": config, "semantics": semantics, "hbm_bytes_per_launch": res,
           "counters_per_launch": counters,
           "lib_sha256": h.hexdigest(), "git_head": git_head(),
           "rule": "2*FETCH_SIZE + WRITE_SIZE (KB->B), per launch, gfx950 wide-read correction",
           "source": summary}, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
