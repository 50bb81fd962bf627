"""Static instruction mix of a kernel in the gfx950 ISA (hipcc -S of
csrc/prk_kernels.hip): instruction classes per loop depth, so the share of
the per-entry setup (depth 1), the row walk (depth 2) and the item loop
(depth 3+) can be read off.  A static count, not a dynamic one: the SQ
counters (tools/sqsum.py) give the executed totals.
usage: python tools/isa_mix.py [kernel-substring] [asm-file]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cpu-renderer_amd")


def asm(path):
    if os.path.exists(path):
        return open(path).read()
    subprocess.run(["make", "-s", "-C", PKG, "asm"], check=True)
    return open(os.path.join(PKG, "build", "prk_kernels.s")).read()


def klass(op):
    if op.startswith("v_div_") or op in ("v_rcp_f32_e32", "v_rcp_f32_e64"):
        return "VALU div/rcp"
    if "_dpp" in op:
        return "VALU dpp"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "VALU lane"
    if op.startswith(("v_cmp", "v_cndmask")):
        return "VALU cmp/select"
    if op.startswith(("v_cvt", "v_rndne", "v_trunc", "v_floor", "v_ceil", "v_fract")):
        return "VALU convert/round"
    if op.startswith(("v_mov", "v_accvgpr")):
        return "VALU move"
    if op.startswith("v_"):
        return "VALU arith"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "SALU/SMEM"
    return "other"


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "k_visILi0ELb1E"
    text = asm(sys.argv[2] if len(sys.argv) > 2 else os.path.join(PKG, "build", "prk_kernels.s"))
    lines = text.splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % want, l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    depth, mix = 0, collections.defaultdict(collections.Counter)
    for l in lines[start:end]:
        m = re.search(r"Depth=(\d+)", l)
        if m and ("Loop Header" in l or "in Loop" in l):
            depth = int(m.group(1))
        elif re.match(r"^\.LBB|^; %bb", l) and "Loop" not in l:
            pass
        s = l.strip()
        if not s or s.startswith((";", ".", "_")):
            continue
        op = s.split()[0]
        mix[depth][klass(op)] += 1
    print("static instruction mix of %s (%s), by loop depth" % (want, lines[start].split(":")[0][:60]))
    total = collections.Counter()
    for d in sorted(mix):
        total.update(mix[d])
        n = sum(mix[d].values())
        print("depth %d: %d instructions" % (d, n))
        for k, v in mix[d].most_common():
            print("   %-20s %6d  %5.1f %%" % (k, v, 100.0 * v / n))
    n = sum(total.values())
    print("all: %d instructions" % n)
    for k, v in total.most_common():
        print("   %-20s %6d  %5.1f %%" % (k, v, 100.0 * v / n))


if __name__ == "__main__":
    main()
