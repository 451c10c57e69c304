#!/usr/bin/env python3
"""Build profiles/pmc_traffic.json (read by bench.py for roofline.traffic)
from the FETCH_SIZE / WRITE_SIZE summaries tools/profile.sh writes.

  python tools/make_traffic.py profiles/r01 > profiles/pmc_traffic.json
"""
import json
import os
import sys


def main():
    d = sys.argv[1].rstrip("/")
    fetch = json.load(open(os.path.join(d, "fetch_summary.json")))
    write = json.load(open(os.path.join(d, "write_summary.json")))
    out = {
        "_round": os.path.basename(d),
        "_source": f"{d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/pmc_run.py "
                   "(tools/profile.sh; cfg3 as bench.py runs it: 4 rotated batches and tables, each measured "
                   "launch on a batch last read > 256 MiB earlier). FETCH_SIZE (KiB) x 1024 x calibration factor, the factor "
                   "measured by a 2 GiB read of known size in each access shape the kernel uses "
                   "(calib_grp<16,4,nt> for 16-lane groups, calib_buf<4,0> for per-lane runs of 4; "
                   "cfg4 weights them by payload share). MI355X_MICROARCH.md section HBM: gfx950 "
                   "under-reports wide streaming reads.",
    }
    for cfg in sorted(k for k in fetch if k.startswith("cfg") and not k.endswith("warm")):
        f = fetch.get(cfg, {})
        if f.get("hbm_bytes_per_launch") is None:
            continue
        w = write.get(cfg, {}).get("avg", {}).get("WRITE_SIZE")
        out[cfg] = {
            "kernel": f.get("kernel"),
            "hbm_bytes_per_launch": f["hbm_bytes_per_launch"],
            "hbm_read_bytes_raw": f["hbm_read_bytes_raw"],
            "fetch_calibration": f["fetch_calibration"],
            "write_bytes": (w * 1024.0) if w is not None else 0.0,
            "algorithmic_bytes": int(f["meta"]["algorithmic_bytes"]),
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
