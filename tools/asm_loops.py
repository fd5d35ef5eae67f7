"""List the loops of a kernel in a hipcc -S listing with their instruction mix.

  python tools/asm_loops.py file.s kernel_substring
"""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):", text, re.M):
        yield m.group(1), m.start()


def main():
    path, sub = sys.argv[1], sys.argv[2]
    text = open(path).read()
    for name, start in kernels(text):
        if sub not in name:
            continue
        end = text.index("s_endpgm", start)
        lines = text[start:end].split("\n")
        labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\w+:", l)}
        print(name)
        for i, l in enumerate(lines):
            m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                body = lines[labels[m.group(1)] : i + 1]
                ins = [re.match(r"\s+([a-z_0-9]+)", b).group(1) for b in body if re.match(r"\s+[a-z_]", b)]
                c = Counter(ins)
                print(f"  loop {m.group(1)}: {len(ins)} instrs; " + ", ".join(f"{k} {v}" for k, v in c.most_common(16)))


if __name__ == "__main__":
    main()
