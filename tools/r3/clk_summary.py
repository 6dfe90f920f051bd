"""Effective clock and MFMA busy per kernel from tools/r3/pmc_clock.sh output:
clk_summary.py <pmc dir> [kernel-trace dir].  GRBM_GUI_ACTIVE is summed over the 8 XCDs:
clock = GRBM / 8 / duration (from the counter rows' own timestamps, or the kernel trace);
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM / 8 x 4 SIMDs x 32 CUs) per XCD."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
rows = defaultdict(dict)
for r in csv.DictReader(open(f)):
    key = (r["Dispatch_Id"], r["Kernel_Name"])
    rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
    rows[key]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = defaultdict(lambda: defaultdict(list))
for (did, name), c in rows.items():
    short = name.split("(")[0].split("::")[-1]
    for k, v in c.items():
        agg[short][k].append(v)
for k, c in agg.items():
    n = len(c["dur"])
    dur = sum(c["dur"]) / n
    g = sum(c.get("GRBM_GUI_ACTIVE", [0])) / n
    mf = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) / n
    clk = g / 8 / dur / 1e9 if dur else 0
    busy = mf / (g / 8 * 4 * 32 * 8) if g else 0
    print(f"{k:28s} n={n:4d} dur={dur*1e6:8.2f} us  clk={clk:5.2f} GHz  mfma_busy={busy:5.3f}")
