"""Static instruction mix of a compiled kernel, per basic block (tuning tool).

    hipcc -O3 --offload-arch=gfx950 ... --cuda-device-only -S -o k.s csrc/kernels_band.hip
    python tools/isa_counts.py k.s 'k_band_phase_resILi1024ELi128ELi16E' [--hist .LBB39_8]

Counts VALU (plain / packed), LDS, vector memory, waits, nops and SALU per block;
--hist prints the opcode histogram of one block (e.g. a kernel's per-row loop body).
DESIGN.md §3 uses these counts with tools/valubench's issue rates for the VALU floor.
"""
import re
import sys


def blocks_of(path, pattern):
    lines = open(path).read().split("\n")
    i0 = next(i for i, l in enumerate(lines) if re.match(r"^_ZN4fcdk\d+" + pattern + r".*:\s*;", l))
    j = i0
    while "s_endpgm" not in lines[j]:
        j += 1
    blocks, cur = [], None
    for l in lines[i0:j + 1]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            cur = [m.group(1), []]
            blocks.append(cur)
            continue
        if cur is None:
            cur = ["entry", []]
            blocks.append(cur)
        s = l.strip()
        if s and not s.startswith(";") and not s.startswith("."):
            cur[1].append(s)
    return blocks


def cls(ins):
    op = ins.split()[0]
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store")):
        return "vmem_st"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    return "salu" if op.startswith("s_") else "other"


def main():
    path, pattern = sys.argv[1], sys.argv[2]
    hist = sys.argv[sys.argv.index("--hist") + 1] if "--hist" in sys.argv else None
    for name, ins in blocks_of(path, pattern):
        c = {}
        for x in ins:
            k = cls(x)
            c[k] = c.get(k, 0) + 1
        br = [x for x in ins if "branch" in x]
        print(name, len(ins), c, br[-2:] if br else "")
        if name == hist:
            h = {}
            for x in ins:
                op = x.split()[0]
                h[op] = h.get(op, 0) + 1
            for k, v in sorted(h.items(), key=lambda a: -a[1]):
                print(f"  {v:5d} {k}")


if __name__ == "__main__":
    main()
