#!/usr/bin/env python3
"""The gfx950 code object a built libs3hash.so ships, and per-kernel facts read from it.

The library's `.hip_fatbin` section is a clang offload bundle; its gfx950 entry is the linked
code object the GPU runs.  Everything here reads THAT object -- not an intermediate `.o` --
so instruction counts (tools/isa_counts.py -> bench.py `issue`), kernel code hashes (the
provenance of profiles/*_pmc.json, bench.py pmc_traffic) and the presence of the device
error-word store (tests/test_code_object.py) describe the shipped code.

    python tools/code_object.py LIB.so [SYMBOL...]   # code hash of each kernel symbol
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FUNC = re.compile(r"^[0-9a-f]+ <(_Z\w+)>:")
LABEL_REF = re.compile(r"\bL[0-9]+\b")


def extract(lib: str, out: str) -> str:
    """Write the gfx950 code object bundled in `lib` to `out`; returns `out`."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.devnull],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", f"--targets={TARGET}", f"--output={out}"],
                       check=True, capture_output=True)
    return out


def kernel_metadata(lib: str) -> dict[str, dict]:
    """{kernel symbol: {private_segment_fixed_size, vgpr_count, vgpr_spill_count, ...}} from the
    shipped code object's AMDGPU metadata note (llvm-readelf --notes)."""
    with tempfile.TemporaryDirectory() as td:
        co = extract(lib, os.path.join(td, "co.o"))
        text = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                              capture_output=True, text=True).stdout
    out, cur = {}, {}
    for line in text.splitlines():
        m = re.match(r"\s*\.(\w+):\s+(\S+)\s*$", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "name" and val.startswith("_Z"):
            cur = out.setdefault(val, {})
        elif key in ("private_segment_fixed_size", "vgpr_count", "sgpr_count",
                     "vgpr_spill_count", "sgpr_spill_count"):  # (keys sorted after .name)
            cur[key] = int(val)
    return out


def disassemble(lib: str, dis_out: str | None = None) -> list[str]:
    """llvm-objdump -d --symbolize-operands of the shipped code object, as lines."""
    with tempfile.TemporaryDirectory() as td:
        co = extract(lib, os.path.join(td, "co.o"))
        text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co],
                              check=True, capture_output=True, text=True).stdout
    if dis_out:
        with open(dis_out, "w") as f:
            f.write(text)
    return text.splitlines()


def function_body(lines: list[str], sym: str) -> list[str]:
    start = next(i for i, l in enumerate(lines) if l.endswith(f"<{sym}>:"))
    end = next((i for i in range(start + 1, len(lines))
                if lines[i].startswith("Disassembly of section") or FUNC.match(lines[i])), len(lines))
    return lines[start + 1:end]


def instructions(body: list[str]) -> list[str]:
    """The kernel's instruction text without addresses and encodings, labels renumbered in
    order of first appearance (llvm-objdump numbers them across the whole file, so another
    kernel's growth would otherwise change this one's text)."""
    out, names = [], {}

    def rename(m):
        return names.setdefault(m.group(0), f"L{len(names)}")

    for l in body:
        if not l.startswith("\t"):
            m = re.match(r"^[0-9a-f]+ <(L[0-9]+)>:", l)
            if m:
                out.append(rename(re.match(r"L[0-9]+", m.group(1))) + ":")
            continue
        ins = l.split("//")[0].strip()
        if ins:
            out.append(LABEL_REF.sub(rename, ins))
    return out


def code_hash(lines: list[str], sym: str) -> str:
    """sha256 (first 16 hex digits) of a kernel's instruction text: the same for any build
    whose machine code for that kernel is the same, whatever else changed in the library."""
    return hashlib.sha256("\n".join(instructions(function_body(lines, sym))).encode()).hexdigest()[:16]


def file_sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


if __name__ == "__main__":
    ls = disassemble(sys.argv[1])
    for s in sys.argv[2:]:
        print(s, code_hash(ls, s))
