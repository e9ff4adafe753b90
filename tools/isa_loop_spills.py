"""Static spill traffic inside one loop of a kernel's ISA (hipcc -S -gline-tables-only output).

  python tools/isa_loop_spills.py <file.s> <kernel symbol substring> <source line in the loop header block>

Finds the kernel's function body, the basic block that carries `.loc 0 <line>` (the loop's
header or a block of it), follows LLVM's '; in Loop: Header=BB..' annotations to every block of
that loop (nested loops included) and counts, per loop depth: instructions, SGPR spill stores
(v_writelane to an 'SGPR spill to VGPR lane' register), spill reloads (v_readlane from one),
s_waitcnt and LDS/global memory instructions."""
import collections
import re
import sys

path, kname, line = sys.argv[1], sys.argv[2], int(sys.argv[3])
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(kname) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
spill_regs = set("v" + r for r in re.findall(r"implicit-def: \$vgpr(\d+) : SGPR spill to VGPR lane", "\n".join(body)))
blocks = []   # label, innermost loop header, depth, parent header (header blocks), instructions
cur = None
for l in body:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(.*)$", l)
    if m:
        lab = m.group(1).replace(".L", "").replace("; %bb.", "BB0_")
        cur = {"label": lab, "header": None, "depth": 0, "parent": None, "ins": [], "locs": set(), "ann": [m.group(2)]}
        blocks.append(cur)
        continue
    if cur is None:
        continue
    s = l.strip()
    if s.startswith(";") and not cur["ins"] and not cur["locs"]:
        cur["ann"].append(s)
        continue
    if s.startswith(".loc"):
        p = s.split()
        if p[1] == "0":
            cur["locs"].add(int(p[2]))
        continue
    if not s or s.startswith((".", ";")):
        continue
    cur["ins"].append(s)
for b in blocks:
    ann = " ".join(b["ann"])
    m = re.search(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)", ann)
    if m:
        b["header"], b["depth"] = m.group(1), int(m.group(2))
    m = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", ann)
    if m:
        b["header"], b["depth"] = b["label"], int(m.group(1))
        par = re.findall(r"Parent Loop (BB\d+_\d+) Depth=(\d+)", ann)
        if par:
            b["parent"] = par[-1][0]
target = [b for b in blocks if line in b["locs"]]
if not target:
    sys.exit(f"no block with .loc 0 {line}")
target.sort(key=lambda b: -b["depth"])
hdr = target[0]["header"] or target[0]["label"]
# the loop = blocks whose header chain reaches hdr: collect headers nested in it
by_label = {b["label"]: b for b in blocks}
def in_loop(b):
    h = b["header"]
    seen = set()
    while h and h not in seen:
        if h == hdr:
            return True
        seen.add(h)
        hb = by_label.get(h)
        h = hb["parent"] if hb else None
    return False
loop = [b for b in blocks if in_loop(b)]
stat = collections.defaultdict(collections.Counter)
for b in loop:
    c = stat[b["depth"]]
    for s in b["ins"]:
        op = s.split()[0]
        c["instr"] += 1
        regs = re.findall(r"\b(v\d+)\b", s)
        if op == "v_writelane_b32" and regs and regs[0] in spill_regs:
            c["spill_store"] += 1
        elif op == "v_readlane_b32" and len(regs) >= 1 and any(r in spill_regs for r in regs):
            c["spill_reload"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("global_"):
            c["global"] += 1
print(f"loop header {hdr}: {len(loop)} blocks; spill VGPRs {sorted(spill_regs)}")
for d in sorted(stat):
    print(f"  depth {d}: {dict(stat[d])}")
