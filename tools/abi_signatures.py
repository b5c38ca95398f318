"""Normalised C prototypes of the engine's public headers (include/crc32c.h,
include/hadoofus_crc32c.h), one per line: `name: return-type name(args)`.

tests/golden/abi_signatures.txt keeps them per ABI version; tests/test_abi.py
checks that the current headers match the current version's section and that
no function kept its name across versions with a different signature (a
changed signature must get a new name, HDFS_CRC32C_ABI_VERSION).

    python tools/abi_signatures.py [header ...]   # print the prototypes"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("crc32c.h", "hadoofus_crc32c.h")]


def prototypes(text):
    """name -> normalised prototype of every function declared in text."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    text = "\n".join(line for line in text.splitlines() if not line.lstrip().startswith("#"))
    text = re.sub(r"typedef\s+struct\s+\w*\s*\{.*?\}\s*\w+\s*;", " ", text, flags=re.S)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b([A-Za-z_]\w*)\s*\(([^;{}()]*)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        if ret.strip() in ("", "return", "sizeof") or name in ("sizeof",):
            continue
        norm = lambda x: re.sub(r"\s*\*\s*", " *", re.sub(r"\s+", " ", x)).strip()
        args = ", ".join(norm(a) for a in args.split(","))
        out[name] = f"{norm(ret)} {name}({args})"
    return out


def header_prototypes(paths=HEADERS):
    out = {}
    for p in paths:
        with open(p) as f:
            out.update(prototypes(f.read()))
    return out


if __name__ == "__main__":
    for name, proto in sorted(header_prototypes(sys.argv[1:] or HEADERS).items()):
        print(f"{name}: {proto}")
