"""Per-kernel register / scratch / spill summary of the product build (gfx950).

    python tools/resources.py [--src mppi_chain.hip] [extra hipcc flags]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"VGPRs": "vgpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "occ", "SGPRs Spill": "sspill", "VGPRs Spill": "vspill"}


def main():
    asm = "/tmp/mppi_res.s"
    args = sys.argv[1:]
    src = "mppi_rocm.hip"
    if args[:1] == ["--src"]:
        src, args = args[1], args[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
           "--cuda-device-only", "-S", "-o", asm, os.path.join(ROOT, "mppi_robotarm_amd/csrc", src),
           "-Rpass-analysis=kernel-resource-usage"] + args
    out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
            cur = {"name": re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+(?:\[[^\]]+\])?): (\d+)", line)
        if m and cur is not None and m.group(1).strip() in KEYS:
            cur[KEYS[m.group(1).strip()]] = m.group(2)
    for r in rows:
        print(f"{r['name']:<40} vgpr {r.get('vgpr', '?'):>4} sgpr {r.get('sgpr', '?'):>4} scratch {r.get('scratch', '?'):>3}"
              f" occ {r.get('occ', '?')} spill s/v {r.get('sspill', '?')}/{r.get('vspill', '?')}")
    print("calls:", open(asm).read().count("s_swappc"))


if __name__ == "__main__":
    main()
