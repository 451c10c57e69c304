"""Summarise a rocprofv3 rocpd database (the default output when no
--output-format is given): per-kernel and per-direction copy statistics, as
JSON.  Usage: python tools/rocpd_summary.py DB [OUT.json]"""

import json
import sqlite3
import sys


def summary(path: str) -> dict:
    c = sqlite3.connect(path)
    kernels = [
        {"name": n, "calls": k, "avg_us": a / 1e3, "min_us": lo / 1e3, "max_us": hi / 1e3, "total_us": t / 1e3}
        for n, k, a, lo, hi, t in c.execute(
            "select name, count(*), avg(end - start), min(end - start), max(end - start), sum(end - start) "
            "from kernels group by name order by sum(end - start) desc")
    ]
    copies = [
        {"direction": n, "copies": k, "avg_us": a / 1e3, "bytes": b, "busy_us": t / 1e3,
         "gb_per_s_while_copying": b / t if t else None}
        for n, k, a, b, t in c.execute(
            "select name, count(*), avg(end - start), sum(size), sum(end - start) from memory_copies group by name")
    ]
    # wall span of each direction's copies (first start to last end): with
    # copies overlapping on several streams, bytes / span is the aggregate rate
    for d in copies:
        lo, hi = c.execute("select min(start), max(end) from memory_copies where name = ?", (d["direction"],)).fetchone()
        d["span_ms"] = (hi - lo) / 1e6
    return {"db": path, "kernels": kernels, "copies": copies}


if __name__ == "__main__":
    s = summary(sys.argv[1])
    text = json.dumps(s, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")
    else:
        print(text)
