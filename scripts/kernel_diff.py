"""Compare one kernel's instruction stream between two gfx950 code objects.

The SHA-256 round code is inline asm whose registers and neighbours the compiler picks, so
a source change anywhere in k_sha256 can move it.  Usage:

  hipcc -O3 -std=c++17 --offload-arch=gfx950 --offload-device-only -c sha256.hip -o a.co
  clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=a.co --output=a.o --unbundle
  llvm-objdump -d --no-show-raw-insn a.o > a.dis          (the same for the other build)
  python scripts/kernel_diff.py a.dis k_sha256E b.dis k_sha256E

prints both instruction counts, the similarity ratio and the number of differing runs
(1.0 / 0: the same code, addresses relative to the kernel's entry)."""
import difflib
import re
import sys


def body(path, name_pat):
    out, inside, start = [], False, 0
    for line in open(path):
        m = re.match(r"^([0-9a-f]+) <(.*)>:", line)
        if m:
            if inside:
                break
            if re.search(name_pat, m.group(2)):
                inside, start = True, int(m.group(1), 16)
            continue
        if inside and line.startswith("\t"):
            m2 = re.match(r"\t(.*?)\s*//\s*([0-9A-Fa-f]+):", line)
            if m2:
                out.append((int(m2.group(2), 16) - start, re.sub(r"<[^>]*>", "", m2.group(1)).strip()))
    return out


def main():
    a, b = body(sys.argv[1], sys.argv[2]), body(sys.argv[3], sys.argv[4])
    sa, sb = [i for _, i in a], [i for _, i in b]
    sm = difflib.SequenceMatcher(None, sa, sb, autojunk=False)
    runs = sum(1 for op in sm.get_opcodes() if op[0] != "equal")
    print(len(a), len(b), "ratio", round(sm.ratio(), 4), "differing runs", runs)


if __name__ == "__main__":
    main()
