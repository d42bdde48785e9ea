"""Per-kernel means of rocprofv3 counter_collection CSVs (all passes under ROOT), agk kernels only."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "agk" not in k:
            continue
        vals[k.split("(")[0][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    m = {c: sum(v) / len(v) for c, v in vals[k].items()}
    print("==", k, " dispatches/counter ~%d" % max(len(v) for v in vals[k].values()))
    for c in sorted(m):
        print("   %-28s %16.0f" % (c, m[c]))
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        print("   wait_any %.1f%%  wait_inst %.1f%%  active %.1f%%" % (
            100 * m.get("SQ_WAIT_ANY", 0) / wc, 100 * m.get("SQ_WAIT_INST_ANY", 0) / wc,
            100 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
        print("   mfma_busy / (gui_active*256CU*4SIMD) = %.1f%%" % (
            100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)))
