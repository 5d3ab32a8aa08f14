"""Register, spill and inline-asm hazard audit of the hand-scheduled kernels
(cdna_hip_programming.md §5.7 item 4).

    python tools/asm_audit.py [-D KEY=VAL ...] [--src FILE.hip ...] [--filter NAME ...]

Compiles csrc/score_scan_bf16.hip, score_scan_f32.hip and mmr.hip (or the
given sources) to gfx950 assembly and checks every score_scan_kernel /
mmr_pick_kernel instantiation:

1. spills: VGPR count, scratch bytes per lane, and the scratch instructions
   and `s_waitcnt vmcnt(0)` between the kernel's first and last MFMA (the hot
   loop; a spill reload there waits vmcnt(0) and drains the LDS-DMA ring);
2. in-flight LDS reads: an inline-asm `ds_read_*` writes its destination
   VGPRs when the data returns, which only the wave's `s_waitcnt lgkmcnt(N)`
   orders; hipcc does not know that, so nothing stops it from reading,
   copying, spilling or reusing those registers in between (round 4's
   cross-pass A prefetch gave wrong lists exactly this way). Every
   instruction between the asm read and the wait that retires it (LDS
   operations return in order: lgkmcnt(N) retires a read once at least N LDS
   operations were issued after it) must not name a destination register;
   a branch or label before the retiring wait is reported too;
3. MFMA results read by inline asm: hipcc inserts the wait states a VALU read
   of an MFMA result needs only in front of its own instructions. An
   inline-asm block that names a register written by an MFMA earlier in the
   straight-line code must have at least the required wait states (other
   instructions, s_nop N = N + 1) in between (round 4's v_max3 asm read
   unfinished MFMA results and gave wrong maxima).
   (LDS-DMA, global_load_lds_*, has no VGPR destination: its address VGPR is
   read at issue, and its LDS bytes are ordered by vmcnt waits and barriers.)

Exit status 0 = clean, 2 = a hazard or a hot-loop spill was found.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diversity-recommendations_amd")
PRODUCT_SOURCES = ("score_scan_bf16", "score_scan_f32", "mmr")
KERNELS = ("score_scan_kernel", "mmr_pick_kernel")

# Wait states between an MFMA's VGPR write and a VALU read of it, gfx950
# (XDL, 16 passes: 32x32 shapes; 8 passes: 16x16). Conservative: the largest.
MFMA_WAIT_STATES = {"32x32": 19, "16x16": 11}
MFMA_LOOKBACK = 64  # instructions searched backward for the MFMA writer

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def compile_asm(src, out, defines=(), extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-munsafe-fp-atomics", f"-I{ROOT}/include", f"-I{PKG}/csrc", "--cuda-device-only",
           "-S", src, "-o", out, *extra] + [f"-D{d}" for d in defines]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return open(out).read()


def functions(text, filt):
    """(name, body lines) of every function whose symbol contains filt."""
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(\S+):\s+; @", text, re.M)]
    for i, (pos, name) in enumerate(starts):
        if filt in name:
            end = starts[i + 1][0] if i + 1 < len(starts) else len(text)
            yield name, text[pos:end].split("\n")


def regs(operands):
    """Set of (file, index) registers named in an operand string."""
    out = set()
    for m in _REG.finditer(operands):
        f = m.group(1)
        if m.group(4) is not None:
            out.add((f, int(m.group(4))))
        else:
            out.update((f, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def instructions(lines):
    """[(line index, mnemonic, operand string, inside inline asm)] of the body."""
    out, in_asm = [], False
    for j, raw in enumerate(lines):
        s = raw.split(";")[0].strip() if ";;#" not in raw else raw.strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(".") or s.startswith(";"):
            continue
        if s.endswith(":"):
            out.append((j, "<label>", s, in_asm))
            continue
        parts = s.split(None, 1)
        out.append((j, parts[0], parts[1] if len(parts) > 1 else "", in_asm))
    return out


def _is_lds(mn):
    return mn.startswith("ds_") and mn not in ("ds_nop",)


def _lgkm_wait(mn, ops):
    if mn != "s_waitcnt":
        return None
    m = re.search(r"lgkmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def inflight_lds_hazards(ins):
    """Instructions that name the destination VGPRs of an inline-asm ds_read
    before the s_waitcnt that retires it (item 2 of the module doc)."""
    bad = []
    for p, (j, mn, ops, in_asm) in enumerate(ins):
        if not (in_asm and mn.startswith("ds_read")):
            continue
        dest = regs(ops.split(",")[0])
        younger = 0
        for (j2, mn2, ops2, _) in ins[p + 1:]:
            n = _lgkm_wait(mn2, ops2)
            if n is not None and n <= younger:
                break  # retired
            if mn2 == "<label>" or mn2.startswith("s_cbranch") or mn2 in ("s_branch", "s_setpc_b64"):
                bad.append((j, j2, f"{mn} {ops}: not retired before {mn2} {ops2}".strip()))
                break
            if _is_lds(mn2):
                younger += 1
            if mn2 != "s_waitcnt" and regs(ops2) & dest:
                bad.append((j, j2, f"{mn} {ops}: in flight when `{mn2} {ops2}` names it"))
                break
    return bad


def _wait_states(mn, ops):
    if mn == "s_nop":
        return int(ops.strip() or 0) + 1
    return 1


def mfma_to_asm_hazards(ins):
    """Inline-asm blocks that name an MFMA result without the wait states
    (item 3 of the module doc)."""
    bad = []
    p = 0
    while p < len(ins):
        if not ins[p][3]:
            p += 1
            continue
        q = p  # one asm block: consecutive in-asm instructions
        named = set()
        while q < len(ins) and ins[q][3]:
            named |= regs(ins[q][2])
            q += 1
        ws = 0
        for (j2, mn2, ops2, in2) in reversed(ins[max(0, p - MFMA_LOOKBACK):p]):
            if mn2 == "<label>":
                continue
            if mn2.startswith("v_mfma"):
                dst = regs(ops2.split(",")[0])
                if dst & named:
                    shape = "16x16" if "16x16" in mn2 else "32x32"
                    if ws < MFMA_WAIT_STATES[shape]:
                        bad.append((j2, ins[p][0], f"asm `{ins[p][1]} {ins[p][2]}` reads `{mn2} "
                                    f"{ops2.split(',')[0]}` after {ws} wait states "
                                    f"(needs {MFMA_WAIT_STATES[shape]})"))
                    break
            elif regs(ops2.split(",")[0]) & named and not mn2.startswith("s_"):
                break  # a non-MFMA writer is closer: the MFMA result is not what asm reads
            ws += _wait_states(mn2, ops2)
        p = q
    return bad


def spill_stats(lines):
    mf = [j for j, l in enumerate(lines) if "v_mfma" in l]
    loop = lines[mf[0]:mf[-1] + 1] if mf else []
    scr = sum(1 for l in loop if "scratch_" in l)
    w0 = sum(1 for l in loop if re.search(r"s_waitcnt\s+vmcnt\(0\)", l))
    return len(mf), scr, w0


def audit_text(text, filters=KERNELS, quiet=False):
    """(hot-loop spills, hazards) over every kernel of the assembly text."""
    spills, hazards = 0, []
    for filt in filters:
        for name, lines in functions(text, filt):
            ins = instructions(lines)
            haz = inflight_lds_hazards(ins) + mfma_to_asm_hazards(ins)
            n_rd = sum(1 for (_, mn, _, a) in ins if a and mn.startswith("ds_read"))
            nmf, scr, w0 = spill_stats(lines)
            meta = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"(.*?)\.end_amdhsa_kernel",
                             text, re.S)
            vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta.group(1)).group(1) if meta else "?"
            sc = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)",
                           meta.group(1)).group(1) if meta else "?"
            if not quiet:
                short = re.sub(r"_ZN\d+dr_\w+?\d+", "", name)[:60]
                print(f"{short:60s} vgpr={vg:>4} scratch={sc:>4} mfma={nmf:3d} "
                      f"loop_scratch={scr:3d} loop_vmcnt0={w0} asm_ds_reads={n_rd:3d} "
                      f"hazards={len(haz)}")
                for h in haz[:5]:
                    print(f"    line {h[0]}->{h[1]}: {h[2]}")
            spills += scr if filt == "score_scan_kernel" else 0
            hazards += [(name,) + h for h in haz]
    return spills, hazards


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--src", action="append", default=[],
                    help="audit these .hip files instead of the product sources")
    ap.add_argument("--filter", action="append", default=[])
    args = ap.parse_args()
    srcs = args.src or [os.path.join(PKG, "csrc", s + ".hip") for s in PRODUCT_SOURCES]
    filters = tuple(args.filter) or KERNELS
    spills, hazards = 0, []
    for src in srcs:
        out = f"/tmp/{os.path.basename(src)}_audit.s"
        try:
            text = compile_asm(src, out, args.defines)
        except RuntimeError as e:
            print(e)
            return 1
        s, h = audit_text(text, filters)
        spills += s
        hazards += h
    print(f"hot-loop spills: {spills}, inline-asm hazards: {len(hazards)}")
    return 0 if spills == 0 and not hazards else 2


if __name__ == "__main__":
    sys.exit(main())
