"""Static instruction mix of the kernels in a gfx950 assembly file (hipcc -S --cuda-device-only).

The chain kernels are fully unrolled (no loops in the layer walk), so the static counts are
the per-wave dynamic counts up to the prologue / composite loops: they price an edit to the
save / split / epilogue code before it goes to the GPU.

    python scripts/isa/isa_mix.py /tmp/chain.s [kernel-substring]
"""
import collections
import re
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith("\t"):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and re.match(r"^\.Lfunc_end", line):
            yield cur, body
            cur, body = None, []
            continue
        if cur:
            body.append(line)


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
            return "valu_dpp"
        if op.startswith("v_permlane"):
            return "valu_permlane"
        if op.startswith("v_cvt"):
            return "valu_cvt"
        if op.startswith("v_fma_mix") or op.startswith("v_mad_mix"):
            return "valu_mix"
        if op.startswith("v_pk_"):
            return "valu_pk"
        if op.startswith("v_accvgpr"):
            return "valu_accmov"
        if op.startswith("v_cndmask") or op.startswith("v_cmp"):
            return "valu_cmp_cnd"
        if op.startswith("v_ldexp"):
            return "valu_ldexp"
        if op.startswith("v_max") or op.startswith("v_min"):
            return "valu_max"
        if op.startswith("v_mov"):
            return "valu_mov"
        if op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("v_writelane"):
            return "valu_lane"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_load_lds") or op.startswith("buffer_load_dword") and "lds" in op:
        return "vmem_dma"
    if op.startswith("global_store") or op.startswith("buffer_store"):
        return "vmem_st"
    if op.startswith("global_") or op.startswith("buffer_"):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_barrier"):
        return "s_barrier"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def mix(body):
    c = collections.Counter()
    ops = collections.Counter()
    for line in body:
        s = line.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        c[classify(op)] += 1
        ops[op] += 1
    return c, ops


if __name__ == "__main__":
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(path):
        if sub not in name:
            continue
        c, ops = mix(body)
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        print(name)
        print("  mfma %d  valu(non-mfma) %d  ratio %.2f" % (c["mfma"], valu, valu / max(1, c["mfma"])))
        for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
            print("   %-16s %6d" % (k, v))
        if "--ops" in sys.argv:
            for k, v in ops.most_common(60):
                print("      %-34s %6d" % (k, v))
