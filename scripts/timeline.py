"""Per-step timeline from a rocprofv3 kernel_trace.csv: busy time, gaps, per-kernel totals for the last N steps."""
import csv, sys, collections
f = sys.argv[1]; steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = [r for r in csv.DictReader(open(f))]
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda t: t[0])
# step boundary = sgd_kernel end
ends = [i for i, k in enumerate(ks) if "sgd_kernel" in k[2]]
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
