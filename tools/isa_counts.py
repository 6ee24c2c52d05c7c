#!/usr/bin/env python3
"""Per-kernel chain-loop instruction counts from the built gfx950 code object (disassembled with
llvm-objdump, so the alignment s_nop the assembler inserts are counted too), written to s3client_amd/kernel_isa_counts.json for bench.py's `issue`
field -- so cycles/instruction is always computed against the shipped code, never a
hand-typed table.

For each kernel the consumer's steady-state loop is the largest loop that is ONE basic block
(a label followed by straight-line code and a branch back to it): the unrolled fast step of
the skew/skewp/quad kernels.  Its instructions (VALU, LDS, SALU, waitcnt, alignment s_nop,
barrier, branch -- everything the wave issues) divided by the blocks one step covers give the
chain instructions per 64-B block.

    llvm-objdump -d --symbolize-operands build/isa/capi-hip-amdgcn-amd-amdhsa-gfx950.o > DIS
    python tools/isa_counts.py DIS OUT.json
"""
import json
import re
import sys

# kernel -> (mangled symbol, 64-B blocks per unrolled consumer step)  (sha256_kernels.hip:
# skew_body kBps = PAIR ? 4 : NC >= 4 ? 2 : 8).  The AUTO kernels up to 28,672 parts; the
# others' consumer loops span several basic blocks and keep hand counts.
KERNELS = {
    "skew": ("_ZN3s3h18sha256_skew_kernelILi1ELb0EEEvNS_10LaunchArgsE", 8),
    "skew_nc2": ("_ZN3s3h18sha256_skew_kernelILi2ELb0EEEvNS_10LaunchArgsE", 8),
    "skewp": ("_ZN3s3h18sha256_skew_kernelILi1ELb1EEEvNS_10LaunchArgsE", 4),
}
INSTR = re.compile(r"^\t([a-z_][a-z0-9_]*)")
LABEL = re.compile(r"^[0-9a-f]+ <(L[0-9]+)>:")
BRANCH = re.compile(r"^\ts_(?:cbranch_\w+|branch)\s+(L[0-9]+)\b")
FUNC = re.compile(r"^[0-9a-f]+ <(_Z\w+)>:")


def function_body(lines, sym):
    start = next(i for i, l in enumerate(lines) if l.endswith(f"<{sym}>:"))
    end = next((i for i in range(start + 1, len(lines))
                if lines[i].startswith("Disassembly of section") or FUNC.match(lines[i])), len(lines))
    return lines[start + 1:end]


def single_block_loops(body):
    """(label, [instruction mnemonics]) for each loop that is one basic block."""
    loops, cur_label, cur = [], None, []
    for l in body:
        m = LABEL.match(l)
        if m:
            cur_label, cur = m.group(1), []
            continue
        mi = INSTR.match(l)
        if not mi:
            continue
        cur.append(mi.group(1))
        mb = BRANCH.match(l)
        if mb:  # a branch ends the basic block
            if cur_label and mb.group(1) == cur_label:
                loops.append((cur_label, list(cur)))
            cur_label, cur = None, []
    return loops


def classify(ops):
    c = {"valu": 0, "lds": 0, "salu": 0, "waitcnt": 0, "nop": 0, "other": 0}
    for op in ops:
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op == "s_nop":
            c["nop"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        else:
            c["other"] += 1
    return c


def main(src, dst):
    lines = open(src).read().splitlines()
    out = {"source": "gfx950 code object of capi.hip, llvm-objdump (tools/isa_counts.py)",
           "kernels": {}}
    for name, (sym, bps) in KERNELS.items():
        loops = single_block_loops(function_body(lines, sym))
        label, ops = max(loops, key=lambda x: len(x[1]))
        c = classify(ops)
        out["kernels"][name] = {
            "symbol": sym, "loop_label": label, "blocks_per_step": bps,
            "instr_per_step": len(ops), "instr_per_block": round(len(ops) / bps, 2),
            "per_block": {k: round(v / bps, 2) for k, v in c.items()},
        }
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    for k, v in out["kernels"].items():
        print(f"{k:9s} {v['instr_per_block']:8.2f} instr/block  {v['per_block']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
