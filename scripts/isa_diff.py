#!/usr/bin/env python3
"""Compare the device ISA of two hipcc -S outputs kernel by kernel (code-motion-free refactors
must leave every kernel's instruction stream unchanged).

    python scripts/isa_diff.py old.s new.s      -> per-kernel: same / differs (+ instruction counts)
"""
import hashlib
import re
import sys


def kernels(path):
    out, name, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name and line.startswith(".Lfunc_end"):
            out[name] = body
            name = None
            continue
        if name:
            s = line.split(";")[0].strip()
            if s and not s.startswith(".") and not s.endswith(":"):
                body.append(re.sub(r"\.L(BB|func_end|tmp)\d+", r".L\1", s))
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    diff = 0
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            print(("only new " if k in b else "only old ") + k)
            diff += 1
            continue
        same = hashlib.sha1("\n".join(a[k]).encode()).digest() == hashlib.sha1("\n".join(b[k]).encode()).digest()
        if not same:
            diff += 1
        print(("same    " if same else "DIFFERS ") + f"{len(a[k]):6d} {len(b[k]):6d} " + k[:100])
    print("ALL SAME" if diff == 0 else f"{diff} kernels differ")
    return 0 if diff == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
