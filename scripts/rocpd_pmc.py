#!/usr/bin/env python3
"""Per-kernel PMC sums (averaged over dispatches) and durations from rocprofv3 rocpd sqlite outputs.
Usage: rocpd_pmc.py DB [DB ...] [--filter SUBSTR]"""
import collections
import sqlite3
import sys


def main(argv):
    flt = None
    if "--filter" in argv:
        i = argv.index("--filter")
        flt = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    out = collections.defaultdict(dict)
    for db in argv:
        con = sqlite3.connect(db)
        q = """select ks.kernel_name, kd.id, kd.start, kd.end, pi.name, sum(pe.value)
               from rocpd_pmc_event pe join rocpd_info_pmc pi on pe.pmc_id = pi.id
               join rocpd_kernel_dispatch kd on kd.event_id = pe.event_id
               join rocpd_info_kernel_symbol ks on kd.kernel_id = ks.id
               group by kd.id, pi.name"""
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        dur = collections.defaultdict(list)
        for kn, did, st, en, cn, v in con.execute(q):
            acc[kn][cn].append(v)
            dur[kn].append((did, en - st))
        for kn in acc:
            if flt and flt not in kn:
                continue
            for cn, vs in acc[kn].items():
                out[kn][cn] = sum(vs) / len(vs)
            ds = {d for d in dur[kn]}
            out[kn]["dur_us"] = sum(x[1] for x in ds) / len(ds) / 1e3
    for kn, cs in out.items():
        print(kn[:100])
        for cn in sorted(cs):
            print(f"   {cn:32s} {cs[cn]:16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
