#!/usr/bin/env python3
"""Turn a tools/profile.sh output directory into profiles/ evidence:
  <tag>_<cfg>_<mode>_kernel_stats.csv   (rocprofv3 --kernel-trace --stats)
  traffic_<cfg>_<mode>.json             (HBM bytes per payload-kernel launch)
written to gpurun_out/evidence/ and then committed under profiles/.
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_unmask_inplace", "k_gather_compact", "k_scatter_compact", "k_unmask_stride", "kb_emit", "k_sspec_pass")
# written under gpurun_out/ (the only directory merged back from the GPU box); copy the
# files into profiles/ to commit them
EVID = os.path.join(REPO, "gpurun_out", "evidence")
os.makedirs(EVID, exist_ok=True)


def counter_rows(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                if any(k in kn for k in KERNELS) and row.get("Counter_Name") == name:
                    vals.append(float(row["Counter_Value"]))
    return vals


def per_kernel(d, name):
    """median counter value per launch of every decode kernel (torch / runtime kernels left out)"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != name or "at::native" in kn or "rocclr" in kn or "k_gen_" in kn:
                    continue
                short = kn.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split()[-1]
                vals.setdefault(short, []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    out, cfg, mode, tag = sys.argv[1:5]
    stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
    avg_ns = None
    if stats:
        dst = os.path.join(EVID, f"{tag}_{cfg}_{mode}_kernel_stats.csv")
        shutil.copy(stats[0], dst)
        with open(stats[0]) as fh:
            for row in csv.DictReader(fh):
                if any(k in row["Name"] for k in KERNELS):
                    avg_ns = float(row["AverageNs"])
    fetch = counter_rows(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = counter_rows(os.path.join(out, "write"), "WRITE_SIZE")
    bench = None
    try:
        with open(os.path.join(out, "bench_trace.json")) as fh:
            bench = json.loads(fh.read().strip().splitlines()[-1])
    except Exception:
        pass
    res = {
        "config": cfg, "mode": mode, "tag": tag,
        "payload_kernel_avg_ns_rocprof": avg_ns,
        "fetch_size_kib_per_launch": statistics.median(fetch) if fetch else None,
        "write_size_kib_per_launch": statistics.median(write) if write else None,
        "launches_counted": [len(fetch), len(write)],
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE reads 1/2)",
    }
    if fetch and write:
        res["hbm_bytes_per_launch"] = int((2 * res["fetch_size_kib_per_launch"]
                                           + res["write_size_kib_per_launch"]) * 1024)
    fk, wk = per_kernel(os.path.join(out, "fetch"), "FETCH_SIZE"), per_kernel(os.path.join(out, "write"), "WRITE_SIZE")
    res["per_kernel_hbm_bytes"] = {k: int((2 * fk[k] + wk.get(k, 0.0)) * 1024) for k in fk}
    res["step_hbm_bytes"] = sum(res["per_kernel_hbm_bytes"].values())
    if bench:
        res["alg_bytes_per_launch"] = bench["roofline"]["alg_bytes_per_launch"]
        res["bench_avg_kernel_us"] = bench["roofline"]["avg_kernel_us"]
        if res.get("hbm_bytes_per_launch"):
            res["traffic_over_alg"] = round(res["hbm_bytes_per_launch"] / res["alg_bytes_per_launch"], 4)
        res["step_traffic_over_alg"] = round(res["step_hbm_bytes"] / res["alg_bytes_per_launch"], 4)
    dst = os.path.join(EVID, f"traffic_{cfg}_{mode}.json")
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
