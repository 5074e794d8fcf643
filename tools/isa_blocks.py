"""VALU / DS / scalar instruction counts per basic block of one kernel's loop (the ISA budget in DESIGN.md §3).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -x hip -S --offload-device-only \
        deequ_amd/csrc/scan.hip -o /tmp/scan.s
    python tools/isa_blocks.py /tmp/scan.s '^_ZN2dq18scan_heavy8_kernelILi2ELb1ELb1ELb1ELb0EEE.*:'

Prints every block inside a loop (Depth >= 2) with its instruction counts and branch targets; the common path of an
iteration is read off by hand (rare branches are the exec-masked NaN / first-batch / zero-rank blocks)."""
import collections
import re
import sys


def main():
    fn, pat = sys.argv[1], sys.argv[2]
    min_depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    lines = open(fn).read().splitlines()
    start = [i for i, l in enumerate(lines) if re.match(pat, l)][0]
    end = start + 1
    while end < len(lines) and not lines[end].startswith(".Lfunc_end"):
        end += 1
    blocks, cur = [], None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\S+|_Z\S+):(.*)", l)
        if m:
            cur = [m.group(1), [], m.group(2)]
            blocks.append(cur)
            continue
        s = l.strip()
        if cur is None or not s or s.startswith(";") or s.startswith("."):
            continue
        cur[1].append(s)
    for name, ins, hdr in blocks:
        depth = int(hdr.split("Depth=")[1].split()[0]) if "Depth=" in hdr else 0
        if depth < min_depth:
            continue
        c = collections.Counter(i.split()[0] for i in ins)
        valu = sum(n for k, n in c.items() if k.startswith("v_"))
        ds = sum(n for k, n in c.items() if k.startswith("ds_"))
        br = [i.split()[0] + " " + i.split()[-1] for i in ins if i.startswith(("s_cbranch", "s_branch"))]
        glob = sum(n for k, n in c.items() if k.startswith(("global_", "buffer_")))
        print("%-12s d%d %4d instr  valu %4d  ds %2d  mem %2d  %s" % (name, depth, len(ins), valu, ds, glob, " ".join(br)))


if __name__ == "__main__":
    main()
