"""Print VGPR / SGPR / scratch / occupancy per kernel of a .hip file (hipcc resource remarks).

    python tools/kernel_resources.py deequ_amd/csrc/scan.hip
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-x", "hip",
           "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
        if not m:
            if "error" in line:
                print(line)
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            name = txt.split(":", 1)[1].strip()
            dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            dm = re.sub(r"\(.*", "", dm).replace("dq::", "")
            cur = {"name": dm}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        print("%-55s vgpr=%-4s sgpr=%-4s scratch=%-4s occ=%-2s lds=%s" % (
            r["name"][:55], r.get("VGPRs"), r.get("TotalSGPRs"), r.get("ScratchSize [bytes/lane]"),
            r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))


if __name__ == "__main__":
    main()
