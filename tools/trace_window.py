"""Per-kernel totals of one window in a rocprofv3 kernel trace: the launches from the N-th
launch of an anchor kernel on (default: the last k_gob_count, i.e. the C5 timed window)."""
import csv
import re
import sys


def main(path, anchor="k_gob_count", which=-1, top=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    i0 = idx[which]
    t0 = int(rows[i0]["Start_Timestamp"])
    agg = {}
    for r in rows[i0:]:
        n = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(n, [0, 0, 1e30, 0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], int(r["Start_Timestamp"]) - t0)
        a[3] = max(a[3], int(r["End_Timestamp"]) - t0)
    for n, a in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print("%-44s %5d %10.2f ms  [%9.2f .. %9.2f]" % (n[-44:], a[0], a[1] / 1e6, a[2] / 1e6, a[3] / 1e6))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
