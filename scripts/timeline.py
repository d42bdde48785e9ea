"""Per-step timeline from a rocprofv3 kernel_trace.csv: busy time, gaps, per-kernel totals for the last N steps."""
import csv, sys, collections
f = sys.argv[1]; steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = [r for r in csv.DictReader(open(f))]
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda t: t[0])
# step boundary = sgd_kernel end
ends = [i for i, k in enumerate(ks) if "sgd_kernel" in k[2] or "sgd_pack_kernel" in k[2]]
if len(ends) < steps + 1:
    print("not enough steps"); sys.exit()
lo, hi = ends[-steps - 1] + 1, ends[-1]
seg = ks[lo:hi + 1]
t0, t1 = seg[0][0], seg[-1][1]
# union of busy intervals
busy, cur_s, cur_e = 0, None, None
for s, e, _ in seg:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("span per step %.3f ms, busy %.3f ms (%.1f%%)" % ((t1 - t0) / steps / 1e6, busy / steps / 1e6, 100 * busy / (t1 - t0)))
tot = collections.defaultdict(float); cnt = collections.Counter()
for s, e, n in seg:
    key = n.split("(")[0][:70]
    tot[key] += (e - s) / 1e3; cnt[key] += 1
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print("  %-70s %6d calls %9.1f us/step" % (k, cnt[k] // steps, v / steps))
# per-queue busy time (main stream vs the wgrad stream) and the serial tail after the last dgrad
qcol = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
if qcol:
    kq = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qcol]) for r in rows),
                key=lambda t: t[0])
    segq = [k for k in kq if t0 <= k[0] <= t1]
    per = collections.defaultdict(float)
    for s, e, n, q in segq:
        per[q] += (e - s) / 1e3
    for q, v in sorted(per.items()):
        print("  queue %-6s kernel time %9.1f us/step" % (q, v / steps))
    # last step: time from the end of the last dgrad (conv_fwd in MODE 3) to the step end
    last = [k for k in segq if k[0] >= ks[ends[-2] + 1][0]]
    dg = [k for k in last if "conv_fwd" in k[2] and (", 3," in k[2] or "Li3E" in k[2] or "<192, 3" in k[2])]
    if dg:
        tail_start = max(e for s, e, n, q in dg)
        print("  serial tail after the last dgrad: %.1f us" % ((last[-1][1] - tail_start) / 1e3))
