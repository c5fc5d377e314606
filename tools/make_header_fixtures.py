"""Writes tests/golden/header_{xor,rs}_doc.txt: the example redundancy-file
headers the reference documents (doc/rst/schemes.rst, XOR example :262-327,
RS example :520-603), with the reST literal-block indent removed. Run here
(the reference is not on the GPU box); the outputs are committed."""
import os
import sys

DOC = "/root/reference/doc/rst/schemes.rst"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def block(lines, first):
    """The literal block starting at 1-based line ``first``."""
    out = []
    for ln in lines[first - 1:]:
        if not ln.strip():
            break
        out.append(ln[2:] if ln.startswith("  ") else ln)
    return "".join(out)


def main():
    with open(DOC) as f:
        lines = f.readlines()
    for name, first in (("xor", 262), ("rs", 520)):
        text = block(lines, first)
        assert text.startswith("CHUNK = "), (name, text[:40])
        with open(os.path.join(OUT, f"header_{name}_doc.txt"), "w") as f:
            f.write(text)
        print(name, len(text.splitlines()), "lines")


if __name__ == "__main__":
    sys.exit(main())
