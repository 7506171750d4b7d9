"""Check on the generated device code that no M0 consumer of the subband kernels reads the
M0 value the slot build leaves behind.

The slot build (dedisperse.hip, build pass) writes M0 with inline asm (``s_mov_b32 m0, ...``
followed by ``s_nop 0``) for its ``ds_write_addtid_b32`` stores and does not restore it,
which is safe only while the compiler writes M0 afresh, in the same basic block, before
every other instruction that reads it.  This walks every basic block of every
``dedisp_sub_kernel`` instantiation and fails if an M0 consumer other than the build's
own stores (LDS-DMA ``global_load_lds*`` / ``buffer_load ... lds``, ``s_movrel*``,
``v_movrel*``, ``s_sendmsg*``, ``ds_gws*``, ``ds_append``, ``ds_consume``,
``ds_read_addtid``) is reached without a compiler-written M0 earlier in its block.

    python scripts/check_m0.py radio-pulsar-utils_amd/csrc/dedisperse-hip-amdgcn-amd-amdhsa-gfx950.s

``__graft_entry__.build()`` runs it on the assembly the production compile keeps
(``-save-temps``, csrc/Makefile) and fails the build on any finding.
"""
import re
import sys

CONSUMERS = ("s_movrel", "v_movrel", "s_sendmsg", "ds_gws", "ds_append", "ds_consume", "ds_read_addtid")


def consumer(op, code):
    return (op.startswith(CONSUMERS) or "global_load_lds" in op
            or (op.startswith("buffer_load") and re.search(r"\blds\b", code) is not None))


def main(path):
    raw = open(path).read().splitlines()
    lines = [ln.split(";")[0].strip() for ln in raw]
    # inline-asm regions (the build's own M0 writes sit between ;;#ASMSTART / ;;#ASMEND;
    # a compiler-written "s_mov_b32 m0 / s_nop 0" pair outside them is the compiler's)
    in_asm, asm = False, []
    for ln in raw:
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
        elif t.startswith(";;#ASMEND"):
            in_asm = False
        asm.append(in_asm)
    text_kernels = 0
    bad = total = 0
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S*dedisp_sub_kernel\S*):$", lines[i])
        if not m:
            i += 1
            continue
        text_kernels += 1
        state = None  # None: unknown, "ours": the build's M0, "cc": compiler-written
        i += 1
        while i < len(lines) and not lines[i].startswith(".Lfunc_end"):
            code = lines[i]
            i += 1
            if not code:
                continue
            if code.endswith(":"):
                state = None  # a new basic block: nothing known about M0
                continue
            op = code.split()[0]
            dst = code.split(",")[0]
            if op.startswith("s_") and re.search(r"\bm0\b", dst) and op not in ("s_sendmsg", "s_sendmsghalt"):
                state = "ours" if asm[i - 1] else "cc"
                continue
            if op.startswith("ds_write_addtid"):
                # the build's own stores (inline asm after its own M0 write; their guarded
                # forms sit in blocks of their own).  They leave the build's M0 behind.
                state = "ours"
                continue
            if consumer(op, code):
                total += 1
                if state != "cc":
                    bad += 1
                    print(f"M0 consumer with M0 {state or 'unset'} in its block:", m.group(1)[:80], code)
    print(f"{text_kernels} subband kernels, {total} M0 consumers, {bad} reading an M0 not written for them")
    return 1 if bad or not total or not text_kernels else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else
                  "radio-pulsar-utils_amd/csrc/dedisperse-hip-amdgcn-amd-amdhsa-gfx950.s"))
