"""Summarise the conv counter passes (scripts/pmc_conv.sh -> gpurun_out/pmc_conv_*, the default
build's kernels; scripts/pmc_x9.sh -> gpurun_out/pmc_x9_*, the exact-split bf16 kernels) of
scripts/conv_pmc.py (CONV_N = 1,024 samples, the learner's [s0; s1]) into profiles/TAG_pmc_conv.txt.
gpurun_out/pmc_f32_* holds an earlier pmc_conv.sh run of the fp32-MFMA conv3 (copied aside).

Per kernel (median over its dispatches of each pass; every pass is its own run):
  wave-cycle split     SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
                       (disjoint, MI355X_MICROARCH.md §rocprofv3 PMC slots)
  MFMA busy            SQ_VALU_MFMA_BUSY_CYCLES / (dispatch duration x 2.4 GHz x 1,024 SIMDs);
                       DVFS lowers the clock under load, so this reads LOW by up to ~15 %
  LDS bank conflicts   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / LDS-array cycles)
  HBM bytes            2 x FETCH_SIZE + WRITE_SIZE (KiB; gfx950 half-counts FETCH_SIZE)
  instructions         SQ_INSTS_MFMA / _VALU / _LDS / _SALU per wave (SQ_WAVES)

    python scripts/summarize_conv_pmc.py TAG
"""
import collections
import csv
import os
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
CLOCK_GHZ, SIMDS = 2.4, 1024


def load(path):
    """{(kernel, grid): {counter: median value, '_us': median duration}}"""
    f = os.path.join(OUT, path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return {}
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "rth::k_conv" not in name or "pack" in name:
            continue
        key = (name.split("(")[0].replace("void ", ""), int(r["Grid_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        vals[key]["_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: {c: st.median(v) for c, v in d.items()} for k, d in vals.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    lines = [__doc__.split("\n\n")[1].strip(), ""]
    for fam, label in (("pmc_conv", "the default build: conv1 bf16x3, conv2 fp32 MFMA, conv3 x9, conv2 dgrad"),
                       ("pmc_f32", "the fp32-MFMA conv3 (RTH_CONV_F32MFMA=1 path; r03 mid-round build)"),
                       ("pmc_x9", "the exact-split bf16 kernels for conv2 (opt-in) and conv3 (scripts/pmc_x9.sh)"),
                       ("pmc_bwd", "the backward kernels at B = 512: x9 data gradients (conv2 classes, conv3) and the "
                                   "x9 weight gradients (scripts/r04.sh bwdpmc)"),
                       ("pmc_fwd", "the torso forward at 1,024 samples: conv1 bf16x3, conv2 fp32 MFMA, conv3 x9 "
                                   "(scripts/r05.sh fwdpmc)")):
        passes = {p: load(f"{fam}_{p}") for p in ("sq", "inst", "fetch", "write", "l2", "ic")}
        keys = sorted(set().union(*[set(d) for d in passes.values()]))
        if not keys:
            continue
        lines.append(f"## {label} ({OUT.split(os.sep)[-1]}/{fam}_*)")
        for k in keys:
            sq, ins = passes["sq"].get(k, {}), passes["inst"].get(k, {})
            fe, wr = passes["fetch"].get(k, {}), passes["write"].get(k, {})
            out = [f"{k[0]}  grid={k[1]}"]
            if sq:
                wc = sq.get("SQ_WAVE_CYCLES", 0) or 1
                out.append(f"  duration {sq['_us']:.1f} us (sq pass); waves: parked {sq.get('SQ_WAIT_ANY', 0) / wc:.0%}, "
                           f"issue-stalled {sq.get('SQ_WAIT_INST_ANY', 0) / wc:.0%} (LDS issue "
                           f"{sq.get('SQ_WAIT_INST_LDS', 0) / wc:.0%}), issuing {sq.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0%}")
                busy = sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (sq["_us"] * 1e3 * CLOCK_GHZ * SIMDS)
                out.append(f"  MFMA busy {busy:.0%} of the SIMD-cycles at {CLOCK_GHZ} GHz")
                if ins.get("SQ_LDS_IDX_ACTIVE"):
                    out.append(f"  LDS bank conflicts {sq.get('SQ_LDS_BANK_CONFLICT', 0) / ins['SQ_LDS_IDX_ACTIVE']:.0%} "
                               "of the LDS-array cycles")
            if ins.get("SQ_WAVES"):
                w = ins["SQ_WAVES"]
                out.append("  per wave: " + ", ".join(f"{c[9:].lower()} {ins.get(c, 0) / w:.0f}" for c in
                                                      ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"))
                           + f" ({w:.0f} waves)")
            if fe and wr:
                out.append(f"  HBM {(2 * fe.get('FETCH_SIZE', 0) + wr.get('WRITE_SIZE', 0)) * 1024 / 1e6:.1f} MB "
                           f"(fetch {2 * fe.get('FETCH_SIZE', 0) * 1024 / 1e6:.1f}, write "
                           f"{wr.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f})")
            l2 = passes["l2"].get(k, {})
            if l2.get("TCC_HIT_sum") is not None:
                h, m = l2.get("TCC_HIT_sum", 0), l2.get("TCC_MISS_sum", 0)
                out.append(f"  L2 hit rate {h / max(h + m, 1):.0%}")
            ic = passes["ic"].get(k, {})
            if ic.get("SQC_ICACHE_HITS") is not None:
                h, m = ic.get("SQC_ICACHE_HITS", 0), ic.get("SQC_ICACHE_MISSES", 0)
                out.append(f"  I-cache hit rate {h / max(h + m, 1):.1%}")
            lines += out
        lines.append("")
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_conv.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(open(path).read())


if __name__ == "__main__":
    main()
