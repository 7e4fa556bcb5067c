"""Per-kernel summary of tools/gpu_attn_pmc.sh's counter passes: effective clock (GRBM_GUI_ACTIVE / 8 / duration),
MFMA-busy fraction, SQ wait / active buckets per wave cycle, instruction mix per MFMA, LDS bank conflicts.

  python tools/attn_sq_summary.py gpurun_out/<tag>
"""
import collections
import csv
import json
import re
import sys


def main():
    base = sys.argv[1].rstrip("/") + "/"
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    dur = collections.defaultdict(list)
    for p in ("pa", "pb", "pc"):
        for r in csv.DictReader(open(base + p + "/p_counter_collection.csv")):
            m = re.search(r"(attn_\w+)(<[^>]*>)?", r["Kernel_Name"])
            if not m:
                continue
            k = m.group(1) + (m.group(2) or "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
            if p == "pc" and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k, d in acc.items():
        m = {c: v / cnt[k][c] for c, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES") or 1.0
        out = {}
        if dur[k]:
            t = sum(dur[k]) / len(dur[k])
            out["launch_us"] = round(t / 1e3, 1)
            out["clock_GHz"] = round(m.get("GRBM_GUI_ACTIVE", 0) / 8 / t, 3)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
            if c in m:
                out[c + "/WAVE_CYCLES"] = round(m[c] / wc, 3)
        if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            out["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] * 8 / (m["GRBM_GUI_ACTIVE"] * 1024), 3)
        if m.get("SQ_INSTS_MFMA"):
            out["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 2)
            out["lds_per_mfma"] = round(m["SQ_INSTS_LDS"] / m["SQ_INSTS_MFMA"], 2)
            out["salu_per_mfma"] = round(m["SQ_INSTS_SALU"] / m["SQ_INSTS_MFMA"], 2)
            out["mfma_insts_M"] = round(m["SQ_INSTS_MFMA"] / 1e6, 2)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            out["lds_bank_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 3)
        res[k] = out
        print(k, json.dumps(out))
    json.dump(res, open(base + "sq_summary.json", "w"), indent=1)


if __name__ == "__main__":
    main()
