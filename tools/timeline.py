"""Prints the GPU timeline (kernels + copies, microseconds from the first event shown) of the last queries of a
rocprofv3 --kernel-trace --memory-copy-trace CSV run.  Usage: timeline.py <dir with run_kernel_trace.csv> [kernel]
[skip] [span]: leave out the last `skip` anchor launches (e.g. the bench's serialized passes) and show `span` periods."""
import csv
import os
import sys


def main(d, anchor="filter_groupby", skip=0, span=2):
    skip, span = int(skip), int(span)
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
    mc = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(mc):
        for r in csv.DictReader(open(mc)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "")))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if anchor in e[2]]
    if len(idx) < span + 1 + skip:
        print("anchor kernel seen %d times" % len(idx))
        return
    lo, hi = idx[-1 - span - skip], idx[-1 - skip]
    t0 = ev[lo][0]
    for e in ev[lo:hi + 1]:
        print("%9.1f %9.1f %8.1f  %s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3, (e[1] - e[0]) / 1e3, e[2]))
    print("period between the last two anchors shown: %.1f us; mean over the %d shown: %.1f us"
          % ((ev[hi][0] - ev[idx[-2 - skip]][0]) / 1e3, span, (ev[hi][0] - ev[lo][0]) / 1e3 / span))


if __name__ == "__main__":
    main(*sys.argv[1:])
