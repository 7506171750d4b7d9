"""Check on the generated device code (make -C radio-pulsar-utils_amd/csrc asm) that every
LDS-DMA instruction of the subband kernels has M0 written earlier in its own basic block:
the slot build writes M0 with inline asm and does not restore it (dedisperse.hip, build
pass), which is safe only while the compiler never carries an M0 value across blocks.

    python scripts/check_m0.py [radio-pulsar-utils_amd/csrc/dedisperse.s]
"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "radio-pulsar-utils_amd/csrc/dedisperse.s"
text = open(path).read()
bad = total = kernels = 0
for m in re.finditer(r"^(_ZN\S*dedisp_sub_kernel\S*):", text, re.M):
    end = text.find(".Lfunc_end", m.end())
    kernels += 1
    m0_set = False
    for line in text[m.end():end].splitlines():
        code = line.split(";")[0].strip()
        if not code:
            continue
        if code.endswith(":"):
            m0_set = False
            continue
        op = code.split()[0]
        if op.startswith("ds_write_addtid"):
            m0_set = False  # M0 holds the slot build's store address (set by inline asm)
        elif op.startswith("s_") and re.search(r"\bm0\b", code.split(",")[0]):
            m0_set = True
        if ("global_load_lds" in op) or (op.startswith("buffer_load") and " lds" in code):
            total += 1
            if not m0_set:
                bad += 1
                print("LDS-DMA without M0 set in its block:", m.group(1)[:80], code)
print(f"{kernels} subband kernels, {total} LDS-DMA instructions, {bad} without M0 set in their block")
sys.exit(1 if bad or not total else 0)
