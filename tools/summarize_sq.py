#!/usr/bin/env python3
"""Condense the SQ counter passes of tools/profile_sq.sh (gpurun_out/prof_sq/p*/) for the
traversal kernel into profiles/<prefix>_sq_summary.md.

Usage: python tools/summarize_sq.py gpurun_out/prof_sq profiles/r01_c3
VALU busy per SIMD = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (256 CUs x 4 SIMDs), against the
kernel length GRBM_GUI_ACTIVE / 8 XCDs (counters summed over the shader engines).
"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = "k_traverse<false, true, "  # both fused-kick variants (1: kick+drift, 2: kick)


def main():
    global KERNEL
    src, prefix = sys.argv[1], sys.argv[2]
    if len(sys.argv) > 3:  # another kernel: print only, the committed files stay the traversal's
        KERNEL = sys.argv[3]
        prefix = "/tmp/sq_other"
    acc = collections.defaultdict(list)  # counter -> per-dispatch totals
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            acc[c].append(v)
    avg = {c: sum(v) / len(v) for c, v in acc.items()}
    waves = avg.get("SQ_WAVES", 0.0)
    config = os.environ.get("CONFIG", "c3")
    out = [f"## {KERNEL.strip(', ')}...> SQ counters ({config.upper()}, average per dispatch; rocprofv3 --pmc, "
           f"{len([d for d in glob.glob(os.path.join(src, 'p*')) if os.path.isdir(d)])} passes)", "",
           "| counter | per dispatch | per wave |", "|---|---|---|"]
    for c in sorted(avg):
        pw = avg[c] / waves if waves else 0.0
        out.append(f"| {c} | {avg[c]:.4g} | {pw:.4g} |")
    if "GRBM_GUI_ACTIVE" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        klen = avg["GRBM_GUI_ACTIVE"] / 8
        busy = avg["SQ_ACTIVE_INST_VALU"] * 4 / 1024
        out += ["", f"- kernel length: GRBM_GUI_ACTIVE / 8 XCDs = {klen:.4g} cycles",
                f"- VALU busy per SIMD: SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs = {busy:.4g} cycles "
                f"= {100 * busy / klen:.1f} % of the kernel"]
    if waves and "SQ_INSTS_VALU" in avg:
        out.append(f"- per wave: VALU {avg['SQ_INSTS_VALU'] / waves:.0f}, SALU "
                   f"{avg.get('SQ_INSTS_SALU', 0) / waves:.0f}, SMEM "
                   f"{avg.get('SQ_INSTS_SMEM', 0) / waves:.0f} instructions")
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        out.append(f"- wave time split: active {100 * avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0f} %, "
                   f"waiting on memory (WAIT_ANY) {100 * avg.get('SQ_WAIT_ANY', 0) / wc:.0f} %, "
                   f"waiting for issue (WAIT_INST_ANY) {100 * avg.get('SQ_WAIT_INST_ANY', 0) / wc:.0f} %")
    if avg.get("SQC_DCACHE_REQ"):
        out.append(f"- scalar data cache: {100 * avg.get('SQC_DCACHE_HITS', 0) / avg['SQC_DCACHE_REQ']:.1f} % "
                   f"hits, {avg.get('SQC_TC_DATA_READ_REQ', 0) / waves if waves else 0:.0f} L2 read "
                   f"requests per wave (SQC_TC_DATA_READ_REQ)")
    if avg.get("TCC_HIT", 0) + avg.get("TCC_MISS", 0):
        out.append(f"- L2 (all requests of the kernel): "
                   f"{100 * avg['TCC_HIT'] / (avg['TCC_HIT'] + avg.get('TCC_MISS', 0)):.1f} % hits")
    open(prefix + "_sq_summary.md", "w").write("\n".join(out) + "\n")
    if KERNEL.startswith("k_traverse") and "GRBM_GUI_ACTIVE" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        path = os.path.join(os.path.dirname(prefix) or ".", "valu_busy.json")
        try:
            doc = json.load(open(path))
        except (OSError, ValueError):
            doc = {}
        doc.setdefault(config, {})["k_traverse"] = {
            "valu_busy": round(busy / klen, 4),
            "valu_insts_per_wave": round(avg.get("SQ_INSTS_VALU", 0) / waves) if waves else None,
            "method": "SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs over GRBM_GUI_ACTIVE / 8 XCDs",
            "source": prefix + "_sq_summary.md",
        }
        json.dump(doc, open(path, "w"), indent=1)
    print("\n".join(out))


if __name__ == "__main__":
    main()
