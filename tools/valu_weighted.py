"""Weighted VALU cycles of a kernel instance: how busy its VALU work keeps the SIMDs.

A wave64 VALU instruction holds a SIMD-32 for a number of cycles that depends on its form:
~2.3-2.5 for f32 add / mul / fma and 32-bit logic, ~4.1-4.5 for integer multiplies, SDWA,
compares, selects with an SGPR mask, conversions, f64 and the div_scale family, ~8.1 for
transcendentals (measured with 8 waves per SIMD: tools/valu_rates.hip ->
profiles/archive/r01_valu_rates.txt, profiles/r03/r03_valu_rates.txt).  The PMC counts the dynamic VALU
instructions per class (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F32, _INT32, _INT64, _CVT,
_{ADD,MUL,FMA,TRANS}_F64; the rest = SQ_INSTS_VALU minus their sum: moves, compares,
selects, lane ops).  A class mixes forms of different cost (INT32: v_xor 2.5, v_mul_lo_u32
4.2), so each class is priced at the mean cost of the kernel's own instructions of that class
in its hot code: the static disassembly of the instance, without the blocks of the IEEE
division / square-root fallbacks (v_div_scale / v_div_fmas / v_div_fixup / v_sqrt_f32 /
v_cmp_class), which the camera-ray-only instances enter only outside the proven domain.

    weighted_cycles = sum_class PMC_count[class] x mean_cost[class]
    weighted_frac   = weighted_cycles / (1024 SIMDs x clock x kernel time)

The bounds price every class at its cheapest / dearest form.
usage: python tools/valu_weighted.py ASM KERNEL_SYMBOL_PREFIX PMC.json [rates.txt ...] > out.json
"""
import json
import re
import sys
from collections import Counter, defaultdict

# cycles per wave64 instruction per SIMD at 8 waves/SIMD (tools/valu_rates.hip), by form
RATE_KEYS = {
    "v_fma_f32": "k_fma", "v_fmac_f32": "k_fmac", "v_fmamk_f32": "k_fmamk", "v_fmaak_f32": "k_fma_lit",
    "v_mul_f32": "k_mul_f32", "v_add_f32": "k_add_f32", "v_sub_f32": "k_sub_f32",
    "v_subrev_f32": "k_sub_f32", "v_max_f32": "k_max_f32", "v_min_f32": "k_max_f32",
    "v_min3_f32": "k_min3", "v_max3_f32": "k_min3", "v_med3_f32": "k_med3",
    "v_rcp_f32": "k_rcp", "v_rsq_f32": "k_rsq", "v_sqrt_f32": "k_sqrt", "v_sin_f32": "k_sin",
    "v_cos_f32": "k_sin", "v_exp_f32": "k_rcp", "v_log_f32": "k_rcp",
    "v_div_scale_f32": "k_div_scale", "v_div_fmas_f32": "k_div_fmas", "v_div_fixup_f32": "k_div_fixup",
    "v_ldexp_f32": "k_ldexp", "v_frexp_exp_i32_f32": "k_frexp_exp", "v_frexp_mant_f32": "k_frexp_exp",
    "v_rndne_f32": "k_rndne", "v_cvt_f32_u32": "k_cvt_f32_u32", "v_cvt_f32_i32": "k_cvt_f32_u32",
    "v_cvt_i32_f32": "k_cvt_i32", "v_cvt_u32_f32": "k_cvt_u32_f32", "v_cvt_f64_f32": "k_cvt_f64_f32",
    "v_cvt_f32_f64": "k_cvt_f32_f64", "v_mul_f64": "k_mul_f64", "v_fma_f64": "k_fma_f64",
    "v_add_f64": "k_fma_f64",
    "v_mul_lo_u32": "k_mul_lo", "v_mul_hi_u32": "k_mul_hi", "v_mul_u32_u24": "k_mul_u24",
    "v_mad_u32_u24": "k_mad_u24", "v_mad_u64_u32": "k_mad_u64", "v_lshl_add_u32": "k_lshl_add",
    "v_add_lshl_u32": "k_lshl_add", "v_lshl_or_b32": "k_lshl_or", "v_and_or_b32": "k_lshl_or",
    "v_or3_b32": "k_lshl_or", "v_xad_u32": "k_lshl_or", "v_bitop3_b32": "k_bitop3",
    "v_xor_b32": "k_xor", "v_or_b32": "k_xor", "v_and_b32": "k_and", "v_not_b32": "k_xor",
    "v_add_u32": "k_add_u32", "v_sub_u32": "k_add_u32", "v_subrev_u32": "k_add_u32",
    "v_add_co_u32": "k_add_u32", "v_addc_co_u32": "k_add_u32", "v_sub_co_u32": "k_add_u32",
    "v_subb_co_u32": "k_add_u32",
    "v_lshrrev_b32": "k_lshr", "v_lshlrev_b32": "k_lshr", "v_ashrrev_i32": "k_lshr",
    "v_min_u32": "k_max_i32", "v_max_u32": "k_max_i32", "v_min_i32": "k_max_i32",
    "v_max_i32": "k_max_i32", "v_min3_u32": "k_min3_u32", "v_max3_i32": "k_min3_u32",
    "v_max3_u32": "k_min3_u32", "v_min3_i32": "k_min3_u32",
    "v_bfe_u32": "k_bfe", "v_bfi_b32": "k_bfi", "v_perm_b32": "k_perm", "v_alignbit_b32": "k_alignbit",
    "v_lshl_add_u64": "k_lshl_add_u64", "v_lshlrev_b64": "k_lshl_add_u64",
    "v_mov_b32": "k_mov", "v_mov_b64": "k_mov_b64", "v_readfirstlane_b32": "k_readfirstlane",
    "v_readlane_b32": "k_readfirstlane", "v_writelane_b32": "k_readfirstlane",
    "v_mbcnt_lo_u32_b32": "k_add_u32", "v_mbcnt_hi_u32_b32": "k_add_u32",
    "v_pk_fma_f32": "k_pk_fma", "v_pk_mul_f32": "k_pk_mul", "v_pk_add_f32": "k_pk_add",
}
# PMC class of a mnemonic (SQ_INSTS_VALU_<class>); None = counted only in SQ_INSTS_VALU
TRANS = {"v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32", "v_exp_f32", "v_log_f32"}


def pmc_class(m):
    if m in TRANS:
        return "TRANS_F32"
    if m.startswith("v_cvt_"):
        return "CVT"
    if m.endswith("_f64"):
        for k in ("ADD", "MUL", "FMA"):
            if f"_{k.lower()}_" in m + "_":
                return f"{k}_F64"
        return None
    if re.match(r"v_(add|sub|subrev)_f32$", m):
        return "ADD_F32"
    if m == "v_mul_f32":
        return "MUL_F32"
    if re.match(r"v_(fma|fmac|fmamk|fmaak|mad|div_fmas)_f32$", m):
        return "FMA_F32"
    if re.search(r"_(u64|i64|b64)$", m) and not m.startswith("v_mov") or m == "v_mad_u64_u32":
        return "INT64"
    if re.search(r"_(u32|i32|b32|u16|i16)$", m) or re.search(r"_u32_u24$", m):
        if m.startswith(("v_cmp", "v_cndmask", "v_mov", "v_readfirstlane", "v_readlane",
                         "v_writelane")):
            return None
        return "INT32"
    return None


def rate_of(m, rates):
    if m.startswith("v_cmp"):
        k = "k_cmp_f32_e32" if "_f32" in m else "k_cmp_u32_e32"
        return rates.get(k, rates.get("k_cmp_lt", 4.3))
    if m.startswith("v_cndmask"):
        return rates.get("k_cnd_sgpr", 4.2)
    k = RATE_KEYS.get(m)
    if k is None or k not in rates:
        return None
    return rates[k]


def load_rates(paths):
    r = {}
    for p in paths:
        for line in open(p):
            mm = re.match(r"(k_\w+)\s+[\d.]+ ms\s+clk [\d.]+ GHz\s+([\d.]+) cycles", line)
            if mm:
                r[mm.group(1)] = float(mm.group(2))
    if "k_mul_lo_mix" in r and "k_add_u32" in r:
        r["k_mul_lo_in_mix"] = r["k_mul_lo_mix"] - r["k_add_u32"]
    return r


def kernel_blocks(asm_path, prefix):
    lines = open(asm_path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.rstrip().endswith(":")
                 or (l.startswith(prefix) and ": ;" in l))
    blocks, cur = [], []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip()
        if re.match(r"^\.?L?BB\d+_\d+:", t) or re.match(r"^\.LBB\d+_\d+:", t):
            if cur:
                blocks.append(cur)
            cur = []
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        cur.append(op)
        if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    return blocks


COLD = ("v_div_scale_f32", "v_div_fixup_f32", "v_div_fmas_f32", "v_sqrt_f32", "v_cmp_class_f32")


def norm(op):
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)


def main(asm, prefix, pmc_path, *rate_paths):
    rates = load_rates(rate_paths or ["profiles/archive/r01_valu_rates.txt"])
    blocks = kernel_blocks(asm, prefix)
    hot = [b for b in blocks if not any(norm(o) in COLD for o in b)]
    static = Counter(o for b in hot for o in b if o.startswith("v_"))
    all_static = Counter(o for b in blocks for o in b if o.startswith("v_"))
    per_class = defaultdict(list)      # class -> [(count, cost, op)]
    unpriced = Counter()
    for op, n in static.items():
        m = norm(op)
        cost = rate_of(m, rates)
        if op.endswith("_sdwa"):
            cost = rates.get("k_xor_sdwa", 4.1)
        if cost is None:
            unpriced[op] += n
            continue
        per_class[pmc_class(m) or "OTHER"].append((n, cost, op))
    pmc = json.load(open(pmc_path))
    med = pmc["median_per_launch"]
    total = med["SQ_INSTS_VALU"]
    classes = ["ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32", "INT32", "INT64", "CVT",
               "ADD_F64", "MUL_F64", "FMA_F64"]
    dyn = {c: med.get(f"SQ_INSTS_VALU_{c}", 0.0) for c in classes}
    dyn["OTHER"] = max(0.0, total - sum(dyn.values()))
    res = {"kernel": pmc.get("kernel"), "asm": asm, "blocks": len(blocks), "hot_blocks": len(hot),
           "static_valu_hot": sum(static.values()), "static_valu_all": sum(all_static.values()),
           "valu_insts_per_launch": total, "classes": {}, "unpriced_static": dict(unpriced)}
    w = lo = hi = 0.0
    for c, n in dyn.items():
        items = per_class.get(c, [])
        cnt = sum(k for k, _, _ in items)
        if cnt:
            mean = sum(k * v for k, v, _ in items) / cnt
            cmin, cmax = min(v for _, v, _ in items), max(v for _, v, _ in items)
        else:
            mean = cmin = cmax = rates.get("k_fma", 2.36)
        res["classes"][c] = {"pmc_per_launch": n, "static_hot": cnt,
                             "mean_cost": round(mean, 3), "min_cost": cmin, "max_cost": cmax,
                             "forms": {op: [k, v] for k, v, op in sorted(items, key=lambda t: -t[0])}}
        w += n * mean
        lo += n * cmin
        hi += n * cmax
    res["weighted_cycles"] = round(w)
    res["weighted_cycles_bounds"] = [round(lo), round(hi)]
    res["mean_cycles_per_valu"] = round(w / total, 3)
    if "kernel_avg_us" in pmc:
        avail = 1024 * 2.4e9 * pmc["kernel_avg_us"] * 1e-6
        res["weighted_frac_at_2.4GHz"] = round(w / avail, 4)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:])
