"""Register / spill audit of the score-scan kernels (cdna_hip_programming.md §5.7 item 4).

    python tools/asm_audit.py [-D KEY=VAL ...]

Compiles csrc/score_scan_bf16.hip and score_scan_f32.hip to gfx950 assembly with the given defines and, for
every score_scan_kernel instantiation, prints the VGPR count, the scratch
bytes per lane, and the scratch instructions and `s_waitcnt vmcnt(0)` found
between the kernel's first and last MFMA (the hot loop). Any scratch access in
that span is a spill whose compiler wait drains the in-flight LDS-DMA ring.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diversity-recommendations_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--filter", default="score_scan_kernel")
    args = ap.parse_args()
    bad = 0
    for src in ("score_scan_bf16", "score_scan_f32"):
        out = f"/tmp/{src}_audit.s"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-munsafe-fp-atomics", f"-I{ROOT}/include", f"-I{PKG}/csrc", "--cuda-device-only",
               "-S", f"{PKG}/csrc/{src}.hip", "-o", out] + [f"-D{d}" for d in args.defines]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stderr)
            return 1
        bad += audit(open(out).read(), args.filter)
    return 0 if bad == 0 else 2


def audit(text, filt):
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\S+):", text, re.M)]
    bad = 0
    for i, (pos, name) in enumerate(starts):
        if filt not in name:
            continue
        end = starts[i + 1][0] if i + 1 < len(starts) else len(text)
        body = text[pos:end]
        lines = body.split("\n")
        mf = [j for j, l in enumerate(lines) if "v_mfma" in l]
        loop = lines[mf[0]:mf[-1] + 1] if mf else []
        scr = sum(1 for l in loop if "scratch_" in l)  # spills inside the MFMA span
        w0 = sum(1 for l in loop if re.search(r"s_waitcnt\s+vmcnt\(0\)", l))
        meta = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"(.*?)\.end_amdhsa_kernel",
                         text, re.S)
        vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta.group(1)).group(1) if meta else "?"
        sc = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)",
                       meta.group(1)).group(1) if meta else "?"
        short = re.sub(r"_ZN7dr_topk\d+", "", name)[:60]
        print(f"{short:60s} vgpr={vg:>4} scratch={sc:>4} mfma={len(mf):3d} "
              f"loop_scratch={scr:3d} loop_vmcnt0={w0}")
        bad += scr
    return bad


if __name__ == "__main__":
    sys.exit(main())
