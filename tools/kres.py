#!/usr/bin/env python
"""Per-kernel register / scratch / occupancy table of the HIP engine for
gfx950, from the compiler's kernel-resource-usage remarks (no GPU needed).

    python tools/kres.py [--filter SUBSTR]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    src = os.path.join(ROOT, "phylostan_amd", "csrc", "phylo_hip.hip")
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O3",
                            "-std=c++17", "-fPIC", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
                            "-I" + os.path.join(ROOT, "include"), "-c", src, "-o", os.path.join(td, "k.o"),
                            "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd=td)
    rows, cur = [], None
    for ln in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?) \[-Rpass", ln)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            cur[k.strip()] = v.strip()
    cols = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
            "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
    print("%-58s %s" % ("kernel", " ".join("%6s" % c.split()[0][:6] + ("sp" if "Spill" in c else "") for c in cols)))
    for row in rows:
        n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", row["name"])[:58]
        if a.filter and a.filter not in n:
            continue
        print("%-58s %s" % (n, " ".join("%8s" % row.get(c, "-") for c in cols)))
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == "__main__":
    main()
