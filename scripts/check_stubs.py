"""Build check: every kernel the host code launches has a device image in the library.

A host object whose embedded gfx950 code object is stale (compiled from an older
signature of a kernel) links fine and fails only at launch time ("Cannot find Symbol"
and an abort inside the HIP runtime).  For every host launch stub
(`...N__device_stub__<kernel>...`) in the shared library, the matching kernel
descriptor (`<kernel>.kd`) must be present among the library's strings.

usage: python3 scripts/check_stubs.py path/to/lib.so [more.so ...]
"""
import re
import sys

STUB = re.compile(rb"^(.*?)(\d+)__device_stub__(.+)$")
STR = re.compile(rb"[\x21-\x7e]{12,}")


def kernel_names(blob):
    names = set()
    stubs = set()
    for m in STR.finditer(blob):
        s = m.group(0)
        i = s.find(b"_Z")
        if i < 0:
            continue
        s = s[i:]
        if b"__device_stub__" in s:
            stubs.add(s)
        elif s.endswith(b".kd"):
            names.add(s[:-3])
    return stubs, names


def check(path):
    with open(path, "rb") as f:
        blob = f.read()
    stubs, names = kernel_names(blob)
    missing = []
    for s in sorted(stubs):
        m = STUB.match(s)
        if not m:
            continue
        n = int(m.group(2)) - len("__device_stub__")
        kern = m.group(1) + str(n).encode() + m.group(3)
        if kern not in names:
            missing.append(kern.decode())
    return len(stubs), missing


def main(argv):
    bad = 0
    for p in argv[1:]:
        n, missing = check(p)
        for k in missing:
            print(f"{p}: no device image for launched kernel {k}", file=sys.stderr)
        print(f"{p}: {n} launch stubs, {len(missing)} without a device image")
        bad += len(missing)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
