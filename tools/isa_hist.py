"""Instruction-class histogram of one function in a gfx950 disassembly (llvm-objdump -d
--no-show-raw-insn), split into straight-line code and the bodies of its loops (backward
branches).  Usage: tools/isa_hist.py <disasm.s> <symbol-substring>"""
import re
import sys
from collections import Counter, OrderedDict

CLASSES = OrderedDict([
    ("mad64", r"^v_mad_(u64_u32|i64_i32)"),
    ("mul32", r"^v_mul_(lo|hi)_u32|^v_mul_u32|^v_mul_hi"),
    ("bpermute", r"^ds_bpermute|^ds_permute|^v_permlane|_dpp"),
    ("cndmask", r"^v_cndmask"),
    ("addc", r"^v_(addc|subb|subbrev)_co"),
    ("add32", r"^v_(add|sub|subrev)_(co_)?u32|^v_add3|^v_(add|sub)_i32|^v_lshl_add|^v_add_lshl"),
    ("add64", r"^v_lshl_add_u64|^v_add_u64|^v_(add|sub)_nc_u64"),
    ("shift_logic", r"^v_(lshr|lshl|ashr)|^v_(and|or|xor|not|bfe|bfi|alignbit|alignbyte|and_or|or3|xor3|and_or_b32|perm)"),
    ("cmp", r"^v_cmp"),
    ("mov", r"^v_mov|^v_accvgpr|^v_readlane|^v_writelane|^v_readfirstlane"),
    ("scratch", r"^scratch_|^buffer_"),
    ("global", r"^global_|^flat_"),
    ("salu", r"^s_(?!waitcnt|nop|cbranch|branch|setpc|swappc|getpc)"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc|getpc)"),
    ("wait", r"^s_(waitcnt|nop)"),
])


def classify(op):
    for k, rx in CLASSES.items():
        if re.search(rx, op):
            return k
    return "v_other" if op.startswith("v_") else "other"


def main(path, sym):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.endswith(">:") and sym in l:
            start = i
            break
    if start is None:
        sys.exit("symbol not found")
    body = []
    for l in lines[start + 1:]:
        if l.endswith(">:"):
            break
        m = re.match(r"\s+(\S+)(.*)//\s*([0-9A-Fa-f]+):(.*)", l)
        if m:
            body.append((int(m.group(3), 16), m.group(1), m.group(2) + m.group(4)))
    addr_idx = {a: i for i, (a, _, _) in enumerate(body)}
    # loops: a branch to an earlier address
    loops = []
    for i, (a, op, rest) in enumerate(body):
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            m = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", rest)
            t = None
            if m:
                # target relative to symbol start
                t = body[0][0] + int(m.group(1), 16)
            if t is not None and t < a and t in addr_idx:
                loops.append((addr_idx[t], i))
    tot = Counter(classify(op) for _, op, _ in body)
    print(f"{sym}: {len(body)} instructions, {len(loops)} backward branches")
    print("  whole:", dict(tot.most_common()))
    for lo, hi in sorted(loops):
        c = Counter(classify(op) for _, op, _ in body[lo:hi + 1])
        n = hi - lo + 1
        if n < 200:
            continue
        print(f"  loop [{lo}..{hi}] {n} instr:", ", ".join(f"{k} {v} ({100*v/n:.0f}%)" for k, v in c.most_common()))
    calls = Counter(re.search(r"<([^>]+)>", r).group(1) if "<" in r else "?" for _, op, r in body if op == "s_swappc_b64")
    calls2 = Counter(r.strip() for _, op, r in body if op.startswith("s_getpc") or "rel32" in r)
    if calls:
        print("  calls:", dict(calls))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
