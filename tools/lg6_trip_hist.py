"""Trip-weighted instruction-class histogram of the 6-lane verdict (mbls_k_fav_verdict_lg6), per
wave (tools/, not product).

Inputs: the gfx950 disassembly of mbls_k_lg6.o (tools/kernel_meta.sh extracts it) and one
rocprofv3 --pmc SQ_INSTS_* pass (tools/pmc_passes.sh, pass "insts") plus the SQ pass's wave count.

Method:
* the final exponentiation is fully determined by the code: x12_pow_xabs runs 63 iterations
  (b = 62..0) of the cyclotomic-squaring path and 5 of them (the set bits of |x| below the top
  one) also take the x12_mul path, whose j loop runs 6 trips; x12_final_exp calls it 5 times and
  runs 9 x12_mul j loops of its own; x12_inv, the Frobenius maps and fp_inv are added once
  (fp_inv's own loop counted once: a lower bound, ~1.3k VALU per extra trip);
* the Miller loop (miller2_trio, 63 iterations whose body takes different branches per bit and
  per pair count) is the residual: measured VALU per wave minus the final exponentiation, with
  the class mix of its loop body;
* the classes (tools/isa_hist.py) are static; VALU = every class but SALU, branches, waits and
  memory.

  python3 tools/lg6_trip_hist.py <lg6.dis> <insts counter_collection.csv> <waves per launch>
"""
import csv
import sys
from collections import Counter, defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import isa_loops as L  # noqa: E402

NON_VALU = {"salu", "branch", "wait", "scratch", "global", "other"}
X_ABS = 0xD201000000010000


def valu(c):
    return sum(v for k, v in c.items() if k not in NON_VALU)


def body_classes(fn, lo, hi):
    return Counter(L.classify(op) for _, op, *_ in fn["body"][lo:hi + 1])


def find(funcs, sub):
    return next(n for n in funcs if sub in n)


def model(dis):
    funcs = L.parse(dis)
    lp = L.loops(dis, ["x12_pow_xabs", "x12_final_exp", "miller2_trio", "x12_inv", "x12_frob", "fp_inv"])
    get = lambda s: lp[find(lp, s)]  # noqa: E731
    pw, fe = get("x12_pow_xabs"), get("x12_final_exp")
    # x12_pow_xabs: loops (sqr path [a..b]), (whole body [a..c]), (x12_mul j loop)
    sq, whole, jl = sorted(pw["loops"], key=lambda l: (l["lo"], l["hi"]))
    set_bits = bin(X_ABS & ((1 << 63) - 1)).count("1")  # taken multiplies for b = 62..0
    mul_path = whole["classes"] - sq["classes"] - jl["classes"]
    per_call = Counter()
    for k, v in sq["classes"].items():
        per_call[k] += 63 * v
    for k, v in mul_path.items():
        per_call[k] += set_bits * v
    for k, v in jl["classes"].items():
        per_call[k] += set_bits * 6 * v
    rest = pw["classes"] - whole["classes"]
    per_call.update(rest)
    pow_total = Counter({k: 5 * v for k, v in per_call.items()})
    # x12_final_exp's own body, its 9 j loops at 6 trips, x12_inv, frob x1, frob2 x2, fp_inv
    fe_total = Counter(fe["classes"])
    for l in fe["loops"]:
        for k, v in l["classes"].items():
            fe_total[k] += 5 * v
    fe_total.update(get("x12_inv")["classes"])
    fe_total.update(get("x12_frob")["classes"])
    for k, v in lp[find(lp, "x12_frob2")]["classes"].items():
        fe_total[k] += 2 * v
    fi = get("fp_inv")
    fe_total.update(fi["classes"])
    miller = get("miller2_trio")
    main = max(miller["loops"], key=lambda l: l["n"])
    return {"pow_xabs": pow_total, "final_exp_rest": fe_total, "miller_body": main["classes"],
            "set_bits": set_bits, "pow_per_call": per_call}


def measured(csv_path, kernel="mbls_k_fav_verdict_lg6"):
    acc = defaultdict(list)
    for r in csv.DictReader(open(csv_path)):
        if r["Kernel_Name"] == kernel:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def pct(c, tot):
    return ", ".join(f"{k} {v / 1e3:.1f}k ({100 * v / tot:.1f}%)" for k, v in c.most_common())


def main(dis, csv_path, waves):
    m = model(dis)
    dyn = measured(csv_path)
    waves = float(waves)
    per_wave = {k: v / waves for k, v in dyn.items()}
    v_tot = per_wave["SQ_INSTS_VALU"]
    print(f"measured per wave ({int(waves)} waves/launch): " +
          ", ".join(f"{k[9:]} {v:,.0f}" for k, v in sorted(per_wave.items())))
    print(f"  VALU_INT64 share {per_wave['SQ_INSTS_VALU_INT64'] / v_tot:.3f}; "
          f"LDS per VALU {per_wave['SQ_INSTS_LDS'] / v_tot:.4f}; SALU per VALU {per_wave['SQ_INSTS_SALU'] / v_tot:.4f}")
    pw, fe = m["pow_xabs"], m["final_exp_rest"]
    pv, fv = valu(pw), valu(fe)
    res = v_tot - pv - fv
    mb = m["miller_body"]
    scale = res / valu(mb)
    mil = Counter({k: v * scale for k, v in mb.items()})
    print(f"\nx12_pow_xabs x5 (63 cyclotomic squarings + {m['set_bits']} x12_mul each; exact trips): "
          f"VALU {pv:,.0f} = {100 * pv / v_tot:.1f}% of the wave's VALU")
    print("   per call:", pct(m["pow_per_call"], sum(m["pow_per_call"].values())))
    print(f"rest of the final exponentiation (x12_mul j loops x6, x12_inv, Frobenius, fp_inv once): "
          f"VALU {fv:,.0f} = {100 * fv / v_tot:.1f}%")
    print(f"Miller loop (residual): VALU {res:,.0f} = {100 * res / v_tot:.1f}% "
          f"(= {scale:.1f} x its static loop body; 63 iterations -> {res / 63:,.0f} VALU per iteration)")
    allc = Counter()
    for c in (pw, fe, mil):
        for k, v in c.items():
            if k not in NON_VALU:
                allc[k] += v
    t = sum(allc.values())
    print("\ntrip-weighted VALU classes, whole verdict:", pct(allc, t))
    mad = allc["mad64"]
    print(f"  mad64 {mad / t:.3f} of VALU (measured VALU_INT64 {per_wave['SQ_INSTS_VALU_INT64'] / v_tot:.3f}: "
          "mad64 plus the 64-bit adds/shifts of the column carries)")
    print(f"  non-mad VALU {t - mad:,.0f} per wave; cutting it by half would take the verdict's VALU by "
          f"{100 * (t - mad) / 2 / t:.0f}%")


if __name__ == "__main__":
    main(*sys.argv[1:4])
