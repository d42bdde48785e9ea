"""Compressed instruction sequence of one kernel in a hipcc -S listing: MFMA / DMA / LDS / wait /
barrier / branch / scratch instructions with runs collapsed -- to check where the compiler put the
MFMAs relative to the barriers and whether the loop spills.
    hipcc -x hip -O3 --offload-arch=gfx950 --cuda-device-only -S conv.hip -o /tmp/conv.s
    python scripts/tools/isa_seq.py /tmp/conv.s conv_wgrad_kernelILi160"""
import sys

KEEP = ("v_mfma", "global_load", "buffer_load", "ds_read", "ds_write", "s_waitcnt", "s_barrier", "s_cbranch",
        "scratch_", "s_setprio")


def main():
    src, pat = sys.argv[1], sys.argv[2]
    s = open(src).read()
    starts = [i for i in range(len(s)) if s.startswith(pat, i)]
    for i in starts:
        line_start = s.rfind("\n", 0, i) + 1
        line = s[line_start:s.find("\n", i)].split(";")[0].strip()
        if not line.endswith(":") or line.startswith(("\t", " ", ".")):
            continue
        j = s.index(".Lfunc_end", i)
        print(line)
        comp = []
        for t in (l.strip().split(";")[0].strip() for l in s[i:j].splitlines()):
            if not t or not (t.startswith(KEEP) or (t.startswith(".LBB") and t.endswith(":"))):
                continue
            op = t.split()[0]
            if comp and comp[-1][0] == op and not op.startswith(("s_waitcnt", ".LBB")):
                comp[-1][1] += 1
            else:
                comp.append([op, 1, t[:70]])
        for op, n, t in comp:
            print(f"  {n:3d} {t if op.startswith(('s_waitcnt', 's_cbranch', 'scratch')) else op}")
        break


if __name__ == "__main__":
    main()
