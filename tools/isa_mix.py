"""Instruction mix / resource usage of one kernel in a hipcc -S device assembly file.
usage: isa_mix.py FILE.s SUBSTRING_OF_MANGLED_NAME [top]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pat = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
names = [n for n in re.findall(r"^(_Z[^:\s]+):", s, re.M) if pat in n]
name = names[0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
body = s[i:j]
c = Counter(re.findall(r"^\s+([vsd]s?_\w+|buffer_\w+|global_\w+)", body, re.M))
print(name, "instructions:", sum(c.values()))
for k, v in c.most_common(top):
    print(f"  {k:32s} {v}")
tail = s[j:j + 4000]
for key in ("NumVgprs", "NumAgprs", "TotalNumVgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
    m = re.search(rf";\s*{key}:\s*(\d+)", s[i - 200:j + 4000])
    m = m or re.search(rf"\.{key.lower()}:\s*(\d+)", tail)
    if m:
        print(f"  {key}: {m.group(1)}")
