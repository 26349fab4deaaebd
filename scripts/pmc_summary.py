"""Per-kernel sums of rocprofv3 PMC counters from its sqlite output (rocpd tables): kernel name, dispatches,
mean duration, and each counter summed over dispatches (divided by dispatch count with --mean)."""
import sqlite3
import sys
from collections import defaultdict


def summary(db, mean=False):
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    pmc = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    disp = {}
    for ev, kid, s, e in c.execute("select event_id, kernel_id, start, end from rocpd_kernel_dispatch"):
        disp[ev] = (names.get(kid, str(kid)), e - s)
    acc = defaultdict(lambda: defaultdict(float))
    cnt, dur = defaultdict(int), defaultdict(float)
    for ev, (k, d) in disp.items():
        cnt[k] += 1
        dur[k] += d
    for ev, pid, v in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        if ev in disp:
            acc[disp[ev][0]][pmc.get(pid, str(pid))] += v
    out = {}
    for k in cnt:
        n = cnt[k]
        out[k] = {"dispatches": n, "mean_ns": dur[k] / n,
                  **{p: (v / n if mean else v) for p, v in sorted(acc[k].items())}}
    return out


if __name__ == "__main__":
    import json
    for db in sys.argv[1:]:
        print(db)
        for k, v in summary(db).items():
            print(" ", k[:80], json.dumps(v))
