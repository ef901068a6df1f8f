"""List loops (backward branches) of a kernel in a gfx950 .s file with their instruction mix.
Developer tool: python tools/loops.py file.s kernel_substring"""
import re, sys, collections
src = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
start = next(i for i, l in enumerate(src) if re.match(r"^_Z\w*%s\w*:" % name, l))
end = next(i for i in range(start, len(src)) if "s_endpgm" in src[i])
body = src[start:end + 1]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
for i, l in enumerate(body):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)|\s+s_branch\s+(\.LBB\w+)", l)
    if not m: continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < i:
        seg = body[labels[tgt]:i + 1]
        ins = [s.split()[0] for s in seg if re.match(r"\s+[vsdgb]\w*_", s)]
        c = collections.Counter(ins)
        print(f"loop {tgt} -> line {i}: {len(ins)} instrs; " + ", ".join(f"{k}:{v}" for k, v in c.most_common(12)))
