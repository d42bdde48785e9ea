"""Per-step durations of one kernel family from a rocprofv3 kernel trace.
Usage: python scripts/step_kernels.py TRACE.csv SUBSTRING [steps]
Steps are delimited by pack_input_kernel launches; prints the step span and
the duration (us) of every matching kernel in launch order."""
import csv
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [k[0] for k in ks if "pack_input" in k[2]]
    for j in range(max(0, len(starts) - 1 - nsteps), len(starts) - 1):
        s0, s1 = starts[j], starts[j + 1]
        durs = [round((k[1] - k[0]) / 1e3, 1) for k in ks if s0 <= k[0] < s1 and sub in k[2]]
        print("step %.3f ms  %s: %s" % ((s1 - s0) / 1e6, sub, durs))


if __name__ == "__main__":
    main()
