#!/usr/bin/env python3
"""Where a kernel's scratch traffic happens: its gfx950 ISA (hipcc --cuda-device-only -S with the
Makefile's flags for the object) split into loops (a backward branch to an earlier label closes a
loop), with the v_mad_u64_u32 and scratch load / store counts of every loop and of the whole
kernel.  A kernel whose frame is spilled only outside its loops pays its scratch once per item,
not once per bit.

    python3 tools/isa_loops.py [kernel-substring ...]   (default: the item-pass kernels)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
BASE = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
        "-I" + os.path.join(ROOT, "hbbft_amd/csrc"), "--cuda-device-only", "-S"]
# object -> (source, flags), as the Makefile builds them
OBJECTS = {
    "hbtc_rlc.p6": ("hbtc_rlc.hip", ["-DHBTC_PART=6", "-DHBTC_INLINE_ALL", "-DHBTC_FQMUL_INLINE"]),
    "hbtc_sig.s1": ("hbtc_sig.hip", ["-DHBTC_SIG_PART=1", "-DHBTC_INLINE_ALL", "-DHBTC_FQMUL_INLINE"]),
    "hbtc_sig.s2": ("hbtc_sig.hip", ["-DHBTC_SIG_PART=2", "-DHBTC_INLINE_ALL", "-DHBTC_FQMUL_SR"]),
    "hbtc_check.c1": ("hbtc_check.hip", ["-DHBTC_CHECK_PART=1", "-DHBTC_GT_INLINE", "-DHBTC_FQMUL_SR"]),
    "hbtc_check.c2": ("hbtc_check.hip", ["-DHBTC_CHECK_PART=2", "-DHBTC_GT_INLINE", "-DHBTC_FQMUL_SR"]),
}


def functions(asm):
    lines = asm.split("\n")
    out, cur, start = {}, None, 0
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            cur, start = m.group(1), i
        elif cur and l.strip().startswith(".Lfunc_end"):
            out[cur] = lines[start:i]
            cur = None
    return out


def report(name, body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    count = lambda seg, pat: sum(1 for l in seg if pat in l)
    rows = [f"{name[:90]}",
            f"  whole kernel: {count(body, 'v_mad_u64_u32')} v_mad_u64_u32, "
            f"{count(body, 'scratch_store')} scratch stores, {count(body, 'scratch_load')} scratch loads (static)"]
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    for a, b in loops:
        seg = body[a:b + 1]
        mads = count(seg, "v_mad_u64_u32")
        if mads == 0 and not count(seg, "scratch_"):
            continue
        rows.append(f"  loop lines {a}-{b}: {mads} v_mad_u64_u32, {count(seg, 'scratch_store')} scratch "
                    f"stores, {count(seg, 'scratch_load')} scratch loads")
    return "\n".join(rows)


def main():
    wanted = sys.argv[1:] or ["k_rlc_decode", "k_rlc_items", "k_sig_decode", "k_sig_items"]
    for obj, (src, flags) in OBJECTS.items():
        with tempfile.NamedTemporaryFile(suffix=".s") as tf:
            subprocess.run([HIPCC] + BASE + flags + [os.path.join(ROOT, "hbbft_amd/csrc", src), "-o", tf.name],
                           check=True, stderr=subprocess.DEVNULL)
            asm = open(tf.name).read()
        for name, body in functions(asm).items():
            if any(w in name for w in wanted):
                print(f"[{obj}] " + report(name, body))


if __name__ == "__main__":
    main()
