#!/usr/bin/env python3
"""Per-kernel chain-loop instruction counts from the gfx950 code object that libs3hash.so ships
(extracted from its offload bundle and disassembled with llvm-objdump, tools/code_object.py, so
the alignment s_nop the assembler inserts are counted too), written to
s3client_amd/kernel_isa_counts.json for bench.py's `issue` field -- so cycles/instruction is
always computed against the shipped code, never a hand-typed table.  The same file records
each kernel's code hash (the provenance key of profiles/*_pmc.json) and, for the
flag-synchronised kernels, the global atomic OR that reports a timed-out wait into the device
error word.

For each kernel the consumer's steady-state loop is the largest loop (a label and a branch
back to it, nested spin loops left out): the unrolled fast step of the skew / skewp kernels.  Its instructions (VALU, LDS, SALU, waitcnt, alignment s_nop,
barrier, branch -- everything the wave issues) divided by the blocks one step covers give the
chain instructions per 64-B block.

    python tools/isa_counts.py s3client_amd/lib/libs3hash.so OUT.json [DIS_OUT]
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from code_object import code_hash, disassemble, file_sha256  # noqa: E402

# kernel -> (mangled symbol, 64-B blocks per unrolled consumer step)  (sha256_kernels.hip:
# skew_body kBps = PAIR ? 4 : NC >= 4 ? 2 : 8).  The AUTO kernels up to 28,672 parts; the
# others' consumer loops span several basic blocks and keep hand counts.
KERNELS = {
    "skew": ("_ZN3s3h18sha256_skew_kernelILi1ELb0EEEvNS_10LaunchArgsE", 8),
    "skew_nc2": ("_ZN3s3h24sha256_skew_pairs_kernelENS_10LaunchArgsE", 8),
    "skewp": ("_ZN3s3h18sha256_skew_kernelILi1ELb1EEEvNS_10LaunchArgsE", 4),
    "skews": ("_ZN3s3h25sha256_skew_shared_kernelENS_10LaunchArgsE", 8),
    "md5-pc": ("_ZN3s3h13md5_pc_kernelILi4EEEvNS_10LaunchArgsE", 4),  # S3H_EXP_MD5_BPS
}
# every kernel a plan can launch (code hashes) and the flag-synchronised ones among them, whose
# timed-out waits must reach the device error word (sha256_kernels.hip flag_wait_ge)
ALL_KERNELS = {
    "lane": "_ZN3s3h18sha256_lane_kernelENS_10LaunchArgsE",
    "pc": "_ZN3s3h16sha256_pc_kernelENS_10LaunchArgsE",
    "pair": "_ZN3s3h18sha256_pair_kernelENS_10LaunchArgsE",
    "quad": "_ZN3s3h18sha256_quad_kernelILi1EEEvNS_10LaunchArgsE",
    "quad_nc2": "_ZN3s3h18sha256_quad_kernelILi2EEEvNS_10LaunchArgsE",
    "skew": KERNELS["skew"][0], "skew_nc2": KERNELS["skew_nc2"][0],
    "skewp": KERNELS["skewp"][0], "skews": KERNELS["skews"][0],
    "md5-pc": "_ZN3s3h13md5_pc_kernelILi4EEEvNS_10LaunchArgsE",
    "md5-pc1": "_ZN3s3h13md5_pc_kernelILi1EEEvNS_10LaunchArgsE",
    "dual_split": "_ZN3s3h22sha256_md5_dual_kernelILb0EEEvNS_10LaunchArgsES1_jPmj",
    "dual_group": "_ZN3s3h23sha256_md5_group_kernelILb1EEEvNS_10LaunchArgsES1_",
    "dual_group_skew": "_ZN3s3h23sha256_md5_group_kernelILb0EEEvNS_10LaunchArgsES1_",
    "dual_group_mixed": "_ZN3s3h29sha256_md5_group_mixed_kernelENS_10LaunchArgsES0_jjjPmj",
}
FLAG_KERNELS = ("skew_nc2", "skews", "dual_group", "dual_group_skew", "dual_group_mixed")
ERR_STORE = re.compile(r"^\t(global|flat|buffer)_atomic_or\b")
INSTR = re.compile(r"^\t([a-z_][a-z0-9_]*)")
LABEL = re.compile(r"^[0-9a-f]+ <(L[0-9]+)>:")
BRANCH = re.compile(r"^\ts_(?:cbranch_\w+|branch)\s+(L[0-9]+)\b")
FUNC = re.compile(r"^[0-9a-f]+ <(_Z\w+)>:")


def function_body(lines, sym):
    start = next(i for i, l in enumerate(lines) if l.endswith(f"<{sym}>:"))
    end = next((i for i in range(start + 1, len(lines))
                if lines[i].startswith("Disassembly of section") or FUNC.match(lines[i])), len(lines))
    return lines[start + 1:end]


def loops(body):
    """(label, [mnemonics]) per loop (a label and a later branch back to it).  Left out:
    instructions of loops nested inside -- in the consumer's fast loop those are the flag spin
    loops of the flag-synchronised kernels, which a wave whose producer is ahead never runs
    (their entry check, outside the nested span, is counted) -- and the cold span a forward
    branch skips to report a timed-out wait into the device error word (its atomic OR), which
    only a faulted launch runs (the branch itself is counted)."""
    ops, label_at, branches = [], {}, []
    for l in body:
        m = LABEL.match(l)
        if m:
            label_at[m.group(1)] = len(ops)
            continue
        mi = INSTR.match(l)
        if not mi:
            continue
        mb = BRANCH.match(l)
        if mb:
            branches.append((len(ops), mb.group(1)))
        ops.append(mi.group(1))
    back = [(label_at[t], i, t) for i, t in branches if t in label_at and label_at[t] <= i]
    cold = [(i + 1, label_at[t] - 1) for i, t in branches
            if t in label_at and label_at[t] > i
            and any(ERR_STORE.match("\t" + ops[k]) for k in range(i + 1, label_at[t]))]
    out = []
    for t, i, name in back:
        inner = [(t2, i2) for t2, i2, _ in back if t <= t2 and i2 < i and (t2, i2) != (t, i)]
        inner += [(a, b) for a, b in cold if t <= a and b < i]
        keep = [ops[k] for k in range(t, i + 1) if not any(t2 <= k <= i2 for t2, i2 in inner)]
        out.append((name, keep))
    return out


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


def main(lib, dst, dis_out=None):
    lines = disassemble(lib, dis_out)
    out = {"source": "gfx950 code object shipped in libs3hash.so, llvm-objdump (tools/isa_counts.py)",
           "library_sha256": file_sha256(lib), "kernels": {},
           "code_hash": {k: code_hash(lines, s) for k, s in ALL_KERNELS.items()},
           "error_word_atomics": {k: sum(bool(ERR_STORE.match(l)) for l in function_body(lines, ALL_KERNELS[k]))
                                  for k in FLAG_KERNELS}}
    for name, (sym, bps) in KERNELS.items():
        # the consumer's loop: reads W+K from LDS, never writes it (ds_write_b128) or touches global memory
        cand = [(n, o) for n, o in loops(function_body(lines, sym))
                if not any(x.startswith(("ds_write_b128", "global_load", "global_store", "buffer_",
                                         "flat_")) for x in o)]
        if name == "md5-pc":
            # the consumer's fast loop (every chain live: no per-lane select) comes first in
            # the code, before the ragged-tail loop that is a few selects longer
            cand = [x for x in cand if sum(o.startswith("v_") for o in x[1]) >= 256 * bps]
            label, ops = cand[0]
        else:
            label, ops = max(cand, key=lambda x: len(x[1]))
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
    main(*sys.argv[1:4])
