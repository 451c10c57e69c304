"""CPU: the counter bookkeeping behind roofline.traffic (tools/pmc_parse.py,
tools/make_traffic.py) on a synthetic rocprofv3 counter CSV: dispatches are
matched to the LABEL lines in order, a label of `kernels=k` takes k
dispatches per launch and reports per-launch sums, FETCH_SIZE is scaled by
the calibration of the named access shape, and WRITE_SIZE passes through."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_pass(d, counter, dispatches):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (name, val) in enumerate(dispatches):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": name, "Counter_Name": counter, "Counter_Value": val})


def test_two_kernel_launch_labels(tmp_path):
    cal = (1 << 31) - 4096
    log = tmp_path / "pmc.log"
    log.write_text(
        f"LABEL calib102 bytes={cal}\n"
        "LABEL cfg2 algorithmic_bytes=1000 payload=900 arena=950 n=10 big_share=1.0\n"
        "LABEL cfg8struct algorithmic_bytes=3000 payload=2900 arena=3100 n=10 kernels=2 shape=calib102\n")
    # FETCH_SIZE in KiB: the calibration read reports half its bytes (factor 2)
    fetch = [("calib_grp", cal / 2048.0)] * 3 + [("nsk::csum_hyb", 1.0)] * 3 + \
            [("nsk::tcp_tx<1>", 1.0), ("nsk::tcp_tx<2>", 0.5)] * 3
    write = [("calib_grp", 0.0)] * 3 + [("nsk::csum_hyb", 0.25)] * 3 + \
            [("nsk::tcp_tx<1>", 0.0), ("nsk::tcp_tx<2>", 0.75)] * 3
    _write_pass(tmp_path / "fetch", "FETCH_SIZE", fetch)
    _write_pass(tmp_path / "write", "WRITE_SIZE", write)
    for k in ("fetch", "write"):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_parse.py"), str(tmp_path / k),
                              str(log)], capture_output=True, text=True, check=True).stdout
        (tmp_path / f"{k}_summary.json").write_text(out)
    s = json.loads((tmp_path / "fetch_summary.json").read_text())
    e = s["cfg8struct"]
    assert e["avg"]["FETCH_SIZE"] == 1.5  # both passes of a launch, per launch
    assert "tcp_tx<1>" in e["kernel"] and "tcp_tx<2>" in e["kernel"]
    assert e["fetch_calibration"]["shape"] == {"calib102": 1.0}
    assert abs(e["hbm_bytes_per_launch"] - 1.5 * 1024 * 2.0) < 1e-6
    t = json.loads(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_traffic.py"), str(tmp_path)],
                                  capture_output=True, text=True, check=True).stdout)
    assert t["cfg8struct"]["write_bytes"] == 0.75 * 1024
    assert t["cfg8struct"]["algorithmic_bytes"] == 3000
    assert "cfg2" not in t or t["cfg2"]["write_bytes"] == 0.25 * 1024
