#!/usr/bin/env python3
"""tools/summarize_pmc.py DIR [KERNEL_SUBSTRING...] -- per-kernel averages (per dispatch) of every counter in the
rocprofv3 --pmc passes under DIR (tools/prof_pmc.sh), plus derived ratios.  Prints one JSON object."""
import csv, glob, json, os, sys
from collections import defaultdict

def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if keys and not any(k in name for k in keys):
                continue
            short = name.split("(")[0][:80]
            acc[short][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for k, m in acc.items():
        per = defaultdict(list)
        for (disp, cn), vals in m.items():
            per[cn].append(sum(vals))   # one dispatch: summed over XCDs / instances
        avg = {cn: sum(v) / len(v) for cn, v in per.items()}
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            wc = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if c in avg:
                    avg[c + "_frac"] = avg[c] / wc
        if "FETCH_SIZE" in avg:
            avg["FETCH_GB_corrected"] = avg["FETCH_SIZE"] * 1024 * 2 / 1e9
        out[k] = avg
    print(json.dumps(out, indent=1, sort_keys=True))

if __name__ == "__main__":
    main()
