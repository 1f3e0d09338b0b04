"""Loops, calls and instruction classes of every function in a gfx950 disassembly (tools/, not
product).  Unlike tools/isa_hist.py this follows the long jumps the compiler emits for branches
beyond the 16-bit range (s_getpc_b64 / s_add_u32 literal / s_setpc_b64) and the calls
(s_swappc_b64), so the Miller loop's back edge inside miller2_trio is found.

  python3 tools/isa_loops.py <disasm> [function-substring ...]

prints, per function: size, class histogram, callees (static call sites) and every back edge
(loop) with its body's size and classes; `loops(path)` returns the same as data for
tools/lg6_trip_hist.py.
"""
import re
import sys
from collections import Counter, OrderedDict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_hist import classify  # noqa: E402

HDR = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
INS = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):(.*)$")


def parse(path):
    """OrderedDict name -> {"start": addr, "body": [(addr, op, operands, encoding + branch target)]}"""
    funcs = OrderedDict()
    cur = None
    for line in open(path):
        line = line.rstrip("\n")
        m = HDR.match(line)
        if m:
            cur = {"start": int(m.group(1), 16), "body": []}
            funcs[m.group(2)] = cur
            continue
        if cur is None:
            continue
        m = INS.match(line)
        if m:
            cur["body"].append((int(m.group(3), 16), m.group(1), m.group(2).strip(), m.group(4)))
    return funcs


def sext32(v):
    return v - (1 << 32) if v & 0x80000000 else v


def pair(reg):
    """key of a 64-bit SGPR pair operand: s[18:19] -> "s18", vcc -> "vcc" """
    m = re.match(r"s\[(\d+):\d+\]", reg)
    return "s" + m.group(1) if m else reg


def lo_reg(reg):
    return "vcc" if reg == "vcc_lo" else reg


def edges(funcs):
    """name -> (branches [(src_addr, dst_addr)], calls [(src_addr, callee)])"""
    by_start = {f["start"]: n for n, f in funcs.items()}
    out = {}
    for name, f in funcs.items():
        br, calls, pc = [], [], {}
        for a, op, rest, tail in f["body"]:
            if op.startswith("s_cbranch") or op == "s_branch":
                m = re.search(r"<([^+>]+)\+0x([0-9a-f]+)>", tail)
                if m and m.group(1) in funcs:
                    br.append((a, funcs[m.group(1)]["start"] + int(m.group(2), 16)))
            elif op == "s_getpc_b64":
                pc[pair(rest)] = a + 4
            elif op == "s_add_u32":
                r = re.match(r"(\w+), (\w+), (0x[0-9a-f]+|-?\d+)$", rest)
                if r and r.group(1) == r.group(2) and lo_reg(r.group(1)) in pc:
                    pc[lo_reg(r.group(1))] += sext32(int(r.group(3), 0) & 0xffffffff)
            elif op in ("s_setpc_b64", "s_swappc_b64"):
                t = pc.get(pair(rest.split(",")[-1].strip()))
                if t is None:
                    continue
                if op == "s_setpc_b64":
                    br.append((a, t))
                else:
                    calls.append((a, by_start.get(t, hex(t))))
        out[name] = (br, calls)
    return out


def loops(path, names=None):
    funcs = parse(path)
    ed = edges(funcs)
    res = OrderedDict()
    for name, f in funcs.items():
        if names and not any(s in name for s in names):
            continue
        body = f["body"]
        idx = {a: i for i, (a, *_) in enumerate(body)}
        br, calls = ed[name]
        lps = []
        for src, dst in br:
            if dst <= src and dst in idx:
                lo, hi = idx[dst], idx[src]
                lcalls = Counter(c for a, c in calls if dst <= a <= src)
                lps.append({"lo": lo, "hi": hi, "n": hi - lo + 1,
                            "classes": Counter(classify(op) for _, op, *_ in body[lo:hi + 1]),
                            "calls": lcalls, "long": not body[idx[src]][1].startswith("s_c")
                            and body[idx[src]][1] != "s_branch"})
        res[name] = {"n": len(body), "classes": Counter(classify(op) for _, op, *_ in body),
                     "calls": Counter(c for _, c in calls), "loops": sorted(lps, key=lambda l: l["lo"])}
    return res


def fmt(c, n):
    return ", ".join(f"{k} {v} ({100 * v / n:.0f}%)" for k, v in c.most_common(8))


def main(path, names):
    for name, r in loops(path, names).items():
        print(f"{name}: {r['n']} instr; {fmt(r['classes'], r['n'])}")
        if r["calls"]:
            print("   calls:", dict(r["calls"]))
        for l in r["loops"]:
            print(f"   loop [{l['lo']}..{l['hi']}] {l['n']} instr{' (long jump)' if l['long'] else ''}: "
                  f"{fmt(l['classes'], l['n'])}" + (f"; calls {dict(l['calls'])}" if l["calls"] else ""))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
