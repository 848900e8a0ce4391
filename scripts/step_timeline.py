"""Per-step kernel timeline from a rocprofv3 kernel trace of bench.py.

Usage: python scripts/step_timeline.py <run_kernel_trace.csv> [first_kernel] [skip] [steps]
A step starts at each dispatch whose name contains first_kernel (default:
the BatchNorm statistics kernel of the update, "bn_cascade_partial").  Every
step gets a one-line summary (span, busy union, kernel count); `steps` steps
after the first `skip` (default 3 after 4: inside bench.py's timed steps,
before its serial breakdown pass) are listed kernel by kernel with start and
end relative to the step start, queue and duration (us).  With the walk on
a side stream it is dispatched just before the step's BatchNorm kernel, so
it is listed at the end of the previous step."""
import csv
import sys


def busy_union(iv):
    tot, ce, gaps = 0, None, []
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                gaps.append(s - ce)
            tot += e - s
            ce = e
        elif e > ce:
            tot += e - ce
            ce = e
    return tot, gaps, ce


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "bn_cascade_partial"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    nsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r["Queue_Id"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    if len(starts) < 2:
        raise SystemExit(f"fewer than two '{first}' dispatches")
    spans = list(zip(starts[:-1], starts[1:]))
    for i, (a, b) in enumerate(spans):
        tot, _, _ = busy_union([(r[0], r[1]) for r in rows[a:b]])
        print(f"step {i:3d}: span {(rows[b][0] - rows[a][0]) / 1e3:7.1f} us, "
              f"busy {tot / 1e3:7.1f} us, {b - a} kernels")
    for a, b in spans[skip:skip + nsteps]:
        t0 = rows[a][0]
        print(f"-- step at {t0}")
        for s, e, name, q in rows[a:b]:
            short = name.split("(")[0].replace("void ", "")[-60:]
            print(f"  q{q:>2} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {short}")
        tot, gaps, ce = busy_union([(r[0], r[1]) for r in rows[a:b]])
        print(f"  span {(rows[b][0] - t0) / 1e3:.1f} us, busy {tot / 1e3:.1f} us, gaps "
              f"{', '.join(f'{g / 1e3:.1f}' for g in gaps)} "
              f"(+ {(rows[b][0] - ce) / 1e3:.1f} before the next step)")


if __name__ == "__main__":
    main()
