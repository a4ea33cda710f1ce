"""Per-basic-block instruction mix of one kernel in a hipcc -S device assembly file (blocks over a size).
usage: isa_blocks.py FILE.s SUBSTRING_OF_MANGLED_NAME [min_instructions]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 60
name = [n for n in re.findall(r"^(_Z[^:\s]+):", s, re.M) if sys.argv[2] in n][0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
blocks, cur, lab = [], [], "entry"
for ln in s[i:j].split("\n"):
    m = re.match(r"^(\.LBB\w+):", ln)
    if m:
        blocks.append((lab, cur))
        lab, cur = m.group(1), []
    elif re.match(r"^\s+[vsdbg]\w+", ln):
        cur.append(ln.strip())
blocks.append((lab, cur))
print(name)
for lab, ins in blocks:
    if len(ins) >= mn:
        c = Counter(x.split()[0] for x in ins)
        print(lab, len(ins), dict(c.most_common(24)))
