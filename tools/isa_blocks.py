"""Per-basic-block VALU census of one kernel in a gfx950 .s dump (tools/isa.sh)."""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^" + pat + r".*:\s*(;.*)?$", l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks, cur, name = [], [], "entry"
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        blocks.append((name, cur)); name, cur = m.group(1), []
        continue
    t = l.strip()
    if t and not t.startswith((";", ".")):
        cur.append(t.split()[0])
blocks.append((name, cur))
tot = collections.Counter()
for n, ins in blocks:
    tot.update(ins)
print("total instrs", sum(tot.values()), "valu", sum(v for k, v in tot.items() if k.startswith("v_")))
for n, ins in sorted(blocks, key=lambda b: -len(b[1]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 6]:
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{n}: {len(ins)} instrs, {valu} valu:", ", ".join(f"{k} {v}" for k, v in c.most_common(18)))

# loops: a branch to an earlier label closes a loop [target, this block]
order = {n: i for i, (n, _) in enumerate(blocks)}
print("loops (header -> latch: blocks, instrs, valu, by-opcode):")
raw = lines[start + 1:end]
bi, brs = 0, []
for l in raw:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        bi = order[m.group(1)]
        continue
    m = re.match(r"\s*s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and order[m.group(2)] <= bi:
        brs.append((order[m.group(2)], bi))
for h, t in sorted(set(brs)):
    c = collections.Counter()
    for n, ins in blocks[h:t + 1]:
        c.update(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"  {blocks[h][0]} -> {blocks[t][0]}: {t - h + 1} blocks, {sum(c.values())} instrs, {valu} valu;",
          ", ".join(f"{k} {v}" for k, v in c.most_common(14)))
