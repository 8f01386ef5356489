"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + PMC HBM traffic).

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md §HBM and
cdna_hip_programming.md §7: FETCH_SIZE / WRITE_SIZE are KiB, collected in
separate --pmc passes; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads, so it is doubled here (an upper estimate for
narrower access patterns, which the guide calls uncalibrated).
usage: python tools/prof_summary.py TAG [WORKLOAD]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "hevc1080"
k1_name = "h2j_k1_recon_h264" if workload.startswith("avc") else "h2j_k1_recon_hevc"
out = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)


def short(name):
    n = name.split("(")[0] if "(" in name and not name.startswith("(") else name
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0]


stats = list(csv.DictReader(open(os.path.join(out, f"prof_{tag}", "stats_kernel_stats.csv"))))
pmc = {}
for kind in ("fetch", "write"):
    p = os.path.join(out, f"pmc_{tag}_{kind}", "pmc_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"].replace("(anonymous namespace)::", ""))
            pmc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
lines = [f"# rocprofv3 summary {tag}", "", "| kernel | calls | avg ms | total % | FETCH_SIZE KiB/launch (raw) | WRITE_SIZE KiB/launch | est. HBM GB/launch (2xFETCH+WRITE) |", "|---|---|---|---|---|---|---|"]
k1 = None
for r in stats:
    k = short(r["Name"].replace("(anonymous namespace)::", ""))
    avg_ms = float(r["AverageNs"]) / 1e6
    f = pmc.get(k, {}).get("FETCH_SIZE")
    w = pmc.get(k, {}).get("WRITE_SIZE")
    fa = sum(f) / len(f) if f else None
    wa = sum(w) / len(w) if w else None
    hbm = (2 * fa + wa) * 1024 / 1e9 if fa is not None and wa is not None else None
    lines.append(f"| {k} | {r['Calls']} | {avg_ms:.3f} | {float(r['Percentage']):.2f} | {fa if fa is None else round(fa)} | {wa if wa is None else round(wa)} | {hbm if hbm is None else round(hbm, 3)} |")
    if k == k1_name:
        k1 = {"avg_ms": avg_ms, "fetch_kib": fa, "write_kib": wa, "hbm_bytes_per_launch": hbm * 1e9 if hbm else None}
open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
if k1:
    k1["tag"] = tag
    k1["kernel"] = k1_name
    json.dump(k1, open(os.path.join(prof, f"pmc_k1_{workload}.json"), "w"), indent=1)
print("\n".join(lines))
