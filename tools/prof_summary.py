"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + PMC HBM traffic).

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md §HBM and
cdna_hip_programming.md §7: FETCH_SIZE / WRITE_SIZE are KiB, collected in
separate --pmc passes; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads, so it is doubled here (an upper estimate for
narrower access patterns, which the guide calls uncalibrated).

K1 ("the dominant kernel") is launched once per chunk per sample type
(uint8 / uint16 instantiations; the one that does not match the batch exits at
once) and per occupancy variant (8 or 16 waves per group); a "launch" here is
one chunk: K1 time and traffic are summed over all K1 dispatches and divided
by the number of chunks (= dispatches of the busier sample type).
usage: python tools/prof_summary.py TAG [WORKLOAD]
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "hevc1080"
k1_base = {"avc1080": "h2j_k1_recon_h264", "mixed": "h2j_k1_recon_"}.get(workload, "h2j_k1_recon_hevc")


def k1_group(k):  # dispatches of one group happen once per chunk (width variants alternate)
    return "h264" if "h264" in k else ("hevc_u16" if "unsigned short" in k else "hevc_u8")
out = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


stats = list(csv.DictReader(open(os.path.join(out, f"prof_{tag}", "stats_kernel_stats.csv"))))
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for kind in ("fetch", "write"):
    p = os.path.join(out, f"pmc_{tag}_{kind}", "pmc_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
lines = [f"# rocprofv3 summary {tag}", "",
         "| kernel | calls | avg ms | total % | FETCH_SIZE KiB/launch (raw) | WRITE_SIZE KiB/launch | est. HBM GB/launch (2xFETCH+WRITE) |",
         "|---|---|---|---|---|---|---|"]
k1_time_ns = 0.0
k1_calls_by_pel = collections.Counter()
k1_time_by_pel = collections.Counter()
for r in stats:
    k = short(r["Name"])
    avg_ms = float(r["AverageNs"]) / 1e6
    f = pmc.get(k, {}).get("FETCH_SIZE")
    w = pmc.get(k, {}).get("WRITE_SIZE")
    fa = sum(f) / len(f) if f else None
    wa = sum(w) / len(w) if w else None
    hbm = (2 * fa + wa) * 1024 / 1e9 if fa is not None and wa is not None else None
    lines.append(f"| {k} | {r['Calls']} | {avg_ms:.3f} | {float(r['Percentage']):.2f} | "
                 f"{fa if fa is None else round(fa)} | {wa if wa is None else round(wa)} | "
                 f"{hbm if hbm is None else round(hbm, 3)} |")
    if k.startswith(k1_base):
        pel = k1_group(k)
        k1_time_ns += float(r["TotalDurationNs"])
        k1_calls_by_pel[pel] += int(r["Calls"])
        k1_time_by_pel[pel] += float(r["TotalDurationNs"])
if k1_calls_by_pel:
    main_pel = max(k1_calls_by_pel, key=k1_calls_by_pel.get)
    chunks = k1_calls_by_pel[main_pel]
    # PMC passes ran their own (shorter) bench; normalise by their own chunk count
    pm_f = [v for k, d in pmc.items() if k.startswith(k1_base) for v in d.get("FETCH_SIZE", [])]
    pm_w = [v for k, d in pmc.items() if k.startswith(k1_base) for v in d.get("WRITE_SIZE", [])]
    pm_chunks_f = sum(len(d.get("FETCH_SIZE", [])) for k, d in pmc.items()
                      if k.startswith(k1_base) and k1_group(k) == main_pel)
    pm_chunks_w = sum(len(d.get("WRITE_SIZE", [])) for k, d in pmc.items()
                      if k.startswith(k1_base) and k1_group(k) == main_pel)
    fa = sum(pm_f) / pm_chunks_f if pm_chunks_f else None
    wa = sum(pm_w) / pm_chunks_w if pm_chunks_w else None
    hbm = (2 * fa + wa) * 1024 if fa is not None and wa is not None else None
    k1 = {"kernel": k1_base, "tag": tag, "chunks": chunks, "avg_ms_per_chunk": k1_time_ns / chunks / 1e6,
          "fetch_kib_per_chunk": fa, "write_kib_per_chunk": wa, "hbm_bytes_per_launch": hbm}
    lines += ["", f"K1 per chunk (all {k1_base} dispatches / {chunks} chunks): "
              f"{k1['avg_ms_per_chunk']:.3f} ms, HBM {hbm / 1e9 if hbm else float('nan'):.3f} GB"]
    json.dump(k1, open(os.path.join(prof, f"pmc_k1_{workload}.json"), "w"), indent=1)
open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
