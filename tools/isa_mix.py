"""Static instruction mix of one kernel in a hipcc --save-temps .s file, per basic block and in
total, by class (VALU transcendental / f64 / packed / cvt / other VALU, MFMA, SALU, VMEM
load / store, LDS, SMEM, waitcnt, readlane / writelane).

    python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--blocks N]

Static counts: a loop body counts once.  Used to see where the episode kernel's VALU goes
(the dynamic totals come from the SQ counters, tools/round_profile.sh)."""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_readlane", "v_readfirstlane")):
        return "readlane"
    if op.startswith("v_writelane"):
        return "writelane"
    if op.startswith("v_"):
        if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
            return "valu_trans"
        if "_f64" in op:
            return "valu_f64"
        if op.startswith("v_pk_"):
            return "valu_pk"
        if op.startswith("v_cvt") or "fma_mix" in op:
            return "valu_cvt"
        if op.startswith(("v_mad_u64", "v_mad_i64", "v_mul_hi", "v_mul_lo", "v_lshl_add_u64", "v_add_co", "v_addc",
                          "v_sub_co", "v_subb", "v_lshlrev_b64", "v_ashrrev_i64", "v_lshrrev_b64")):
            return "valu_int64ish"
        if op.startswith(("v_bitop3", "v_xor", "v_and", "v_or", "v_lshl", "v_lshr", "v_ashr", "v_bfe", "v_bfi",
                          "v_alignbit", "v_perm")):
            return "valu_bit"
        if op.startswith(("v_cndmask", "v_cmp", "v_cmpx")):
            return "valu_cmp_sel"
        if op.startswith(("v_mov", "v_accvgpr")):
            return "valu_mov"
        return "valu_other"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_st"
    if op.startswith(("global_atomic", "buffer_atomic", "flat_atomic")):
        return "vmem_atomic"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernel_lines(path, name):
    lines, on = [], False
    for ln in open(path):
        if not on:
            if re.match(r"^[_A-Za-z0-9.$]+:\s*(;.*)?$", ln) and name in ln and not ln.startswith("."):
                on = True
            continue
        if ln.startswith(".Lfunc_end") or re.match(r"^\s*\.size\s", ln):
            break
        lines.append(ln.rstrip("\n"))
    return lines


def main():
    path, name = sys.argv[1], sys.argv[2]
    nblocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 0
    lines = kernel_lines(path, name)
    if not lines:
        sys.exit(f"kernel matching {name!r} not found")
    total = collections.Counter()
    blocks, cur, label = [], collections.Counter(), "entry"
    for ln in lines:
        m = re.match(r"^(\.LBB[0-9_]+):", ln)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), collections.Counter()
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        c = classify(op)
        total[c] += 1
        cur[c] += 1
    blocks.append((label, cur))
    valu = sum(v for k, v in total.items() if k.startswith("valu") or k in ("readlane", "writelane"))
    print(f"{name}: {sum(total.values())} instructions, VALU {valu} (readlane/writelane incl.)")
    for k, v in total.most_common():
        print(f"  {k:16s} {v}")
    if nblocks:
        print("\nlargest blocks:")
        for label, c in sorted(blocks, key=lambda b: -sum(b[1].values()))[:nblocks]:
            print(f"  {label:14s} {sum(c.values()):5d}  " + " ".join(f"{k}={v}" for k, v in c.most_common(8)))


if __name__ == "__main__":
    main()
