"""Summarise rocprofv3 counter_collection CSVs: mean per dispatch of each counter for agk kernels."""
import csv, glob, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for k in sorted(glob.glob(root + "/*")):
    vals = collections.defaultdict(list)
    durs = []
    for f in glob.glob(k + "/*/runc/*_counter_collection.csv") + glob.glob(k + "/*/*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "agk" not in r.get("Kernel_Name", ""):
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(k + "/p1/*/*_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if "agk" in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("==", k.split("/")[-1], "dur_us(median)=%.1f" % (sorted(durs)[len(durs)//2] if durs else 0))
    m = {c: sum(v) / len(v) for c, v in vals.items()}
    for c in sorted(m):
        print("   %-28s %16.0f" % (c, m[c]))
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        wc = m["SQ_WAVE_CYCLES"]
        print("   wait_any %.1f%%  wait_inst %.1f%%  active %.1f%%" % (100*m.get("SQ_WAIT_ANY",0)/wc, 100*m.get("SQ_WAIT_INST_ANY",0)/wc, 100*m.get("SQ_ACTIVE_INST_ANY",0)/wc))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        print("   mfma_busy / (gui_active*256CU*4SIMD) = %.1f%%" % (100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4) ))
    if durs and "GRBM_GUI_ACTIVE" in m:
        print("   effective clock GHz = %.2f" % (m["GRBM_GUI_ACTIVE"] / 8 / (sorted(durs)[len(durs)//2] * 1e3)))
