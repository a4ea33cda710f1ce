"""Print the basic block of a kernel with the most occurrences of an instruction (default v_exp).
usage: isa_block.py FILE.s NAME_SUBSTRING [instr] [rank]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
ins = sys.argv[3] if len(sys.argv) > 3 else "v_exp"
rank = int(sys.argv[4]) if len(sys.argv) > 4 else 0
name = [n for n in re.findall(r"^(_Z[^:\s]+):", s, re.M) if pat in n][0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
blocks, cur, lab = [], [], "entry"
for ln in s[i:j].split("\n"):
    if re.match(r"^\.LBB\S+:", ln):
        blocks.append((lab, cur))
        lab, cur = ln, []
    else:
        cur.append(ln)
blocks.append((lab, cur))
blocks.sort(key=lambda b: -sum(ins in l for l in b[1]))
lab, body = blocks[rank]
code = [l for l in body if l.strip() and not l.strip().startswith(";") and not l.strip().startswith(".")]
print(lab, len(code), "instructions")
print("\n".join(code))
