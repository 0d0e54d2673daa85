"""Summarise rocprofv3 outputs (gpurun_out/) into profiles/ (committed evidence).

    python scripts/summarize_profile.py TAG [--steps N]

Reads gpurun_out/prof/run_kernel_{stats,trace}.csv (rocprofv3 --kernel-trace --stats) and
gpurun_out/pmc_{fetch,write}/run_counter_collection.csv (separate --pmc FETCH_SIZE /
WRITE_SIZE passes), writes
    profiles/TAG_kernel_stats.csv        rocprofv3's own --stats table
    profiles/TAG_steady_state.txt        per-iteration kernel breakdown (timed window)
    profiles/TAG_gather_launches.txt     the learner gather's launches by grid (avg duration)
    profiles/TAG_conv{2,3}_launches.txt  conv2 / conv3 forward launches by grid (conv3: the dominant kernel)
    profiles/TAG_pmc.txt                 FETCH/WRITE per kernel and grid, gfx950-corrected
    profiles/traffic_TAG.json            HBM bytes per launch of the learner gather and of the learner's
                                         conv2 / conv3 (bench.py cites it)
FETCH_SIZE on gfx950 reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md
§HBM): it is doubled; WRITE_SIZE is exact for 16-byte stores.  Both are in KiB.
"""
import collections
import csv
import json
import os
import shutil
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
# learner gather launch (k_copy_rows flat grid): B rows x 2 frame columns x 7 chunks of 4 KiB
# + the small columns one lane per 4-byte word, 256 threads per workgroup
def copy_grid(rows):
    """k_copy_rows' grid (threads) for `rows` apex rows: 2 frame columns x 7 chunks of 4 KiB per
    row + the small columns' workgroups (rows / 64), 256 lanes each"""
    return (rows * 14 + rows // 64) * 256


def copy_grid_fs(rows):
    """k_copy_rows' grid for `rows` frame-store apex rows (the insert: five small columns -- two
    16-byte frame-id tuples, a, r, done -- each a lane per 4-byte word, 256 lanes per workgroup)"""
    return sum((rows * (nb // 4) + 255) // 256 for nb in (16, 8, 4, 16, 4)) * 256


LEARNER_GATHER_GRID = copy_grid(512)
# the HBM-bound kernels of bench.py's roofline_hbm: name -> (kernel-name match, grid or None)
HBM_KERNELS = {"k_tree_update_sub": ("k_tree_update_sub", None), "k_tree_sample": ("k_tree_sample", None),
               "k_copy_rows (gather)": ("k_copy_rows", "gather"), "k_copy_rows (insert)": ("k_copy_rows", "insert"),
               "k_actor_tail": ("k_actor_tail", None), "k_td_heads_backward": ("k_td_heads_backward", None),
               "k_adam": ("k_adam", None), "k_grad_sqsum": ("k_grad_sqsum", None),
               "rth_clip_adam (k_clip_adam_fused)": ("k_clip_adam_fused", None)}
# output bytes per sample of the conv forwards (float32): conv2 writes [81 pixels x 64] NHWC,
# conv3 [64 x 49] NCHW -- a dispatch's WRITE_SIZE says how many samples it ran (the grid does
# not: the conv kernels loop over the samples)
CONV_OUT_BYTES = {"conv2": 81 * 64 * 4, "conv3": 49 * 64 * 4}
# conv2 / conv3 forward: the fp32-MFMA kernel or the exact-split bf16 one (k_conv_x9)
CONV2 = ("k_conv_bias_relu<0, 4, 4, 2, 32, 64, 20, 20", "k_conv_x9<4, 4, 2, 32, 20, 20")
CONV3 = ("k_conv_bias_relu<0, 3, 3, 1, 64, 64, 9, 9", "k_conv_x9<3, 3, 1, 64, 9, 9")


def is_conv(pats, name):
    return any(p in name for p in pats)


def tree_pmc(dirs):
    """--tree-pmc DIR...: k_tree_sample's FETCH_SIZE per dispatch (x2, gfx950) by grid, one line
    per variant directory (scripts/r04.sh treepmc)"""
    for d in dirs:
        p = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(p):
            print(d, "no counters")
            continue
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == "FETCH_SIZE" and "k_tree_sample" in r["Kernel_Name"]:
                by[int(r["Grid_Size"])].append(2 * float(r["Counter_Value"]) * 1024)
        for g, v in sorted(by.items()):
            print(f"{os.path.basename(d):>16} grid={g:>7d} n={len(v):5d} fetch_MB median={st.median(v) / 1e6:.3f} "
                  f"min={min(v) / 1e6:.3f} max={max(v) / 1e6:.3f}")


def main():
    if sys.argv[1] == "--tree-pmc":
        return tree_pmc(sys.argv[2:])
    tag = sys.argv[1]
    arg = lambda k, d: int(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else d
    steps = arg("--steps", 100)
    grids = {"gather": copy_grid(arg("--batch", 512)), "insert": copy_grid(arg("--actors", 256))}
    inloop, loop_grid = {}, {}
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, "prof", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    trace = os.path.join(OUT, "prof", "run_kernel_trace.csv")
    if os.path.exists(trace):
        rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
        ts = [r for r in rows if "k_tree_sample" in r["Kernel_Name"]]
        start = int(ts[-steps]["Start_Timestamp"])  # one PER sample per iteration
        # ... up to the last learner update (the bench's isolated gather / conv timings follow)
        end = max(int(r["End_Timestamp"]) for r in rows if "k_adam" in r["Kernel_Name"] or
                  "k_clip_adam_fused" in r["Kernel_Name"])
        win = [r for r in rows if start <= int(r["Start_Timestamp"]) <= end]
        agg = collections.defaultdict(lambda: [0, 0])
        for r in win:
            a = agg[r["Kernel_Name"][:100]]
            a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            a[1] += 1
        busy = sum(v[0] for v in agg.values())
        learner_stream = next((r.get("Stream_Id") for r in reversed(win) if "k_adam" in r["Kernel_Name"] or
                               "k_clip_adam_fused" in r["Kernel_Name"]), None)
        with open(os.path.join(PROF, f"{tag}_steady_state.txt"), "w") as f:
            f.write(f"# last {steps} iterations of the profiled bench run\n")
            f.write(f"window {((end - start) / 1e6):.3f} ms, kernel-busy {busy / 1e6:.3f} ms, "
                    f"{(end - start) / 1e3 / steps:.1f} us/iter wall, {busy / 1e3 / steps:.1f} us/iter busy, "
                    f"{len(win) / steps:.1f} kernels/iter\n")
            f.write(f"{'share':>7} {'us/iter':>9} {'calls/iter':>10}  kernel\n")
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0]):
                f.write(f"{v[0] / busy * 100:6.2f}% {v[0] / 1e3 / steps:9.2f} {v[1] / steps:10.2f}  {k}\n")
        for name, (match, g) in HBM_KERNELS.items():  # in-loop mean launch durations (bench.py roofline_hbm)
            sel = [r for r in win if match in r["Kernel_Name"]
                   and (g is None or int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) == grids[g])]
            if not sel and g == "insert":  # the frame-store insert (frame ids, not stacks)
                grids[g] = copy_grid_fs(arg("--actors", 256))
                sel = [r for r in win if match in r["Kernel_Name"]
                       and int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) == grids[g]]
            if sel:
                inloop[name] = round(st.mean(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel) / 1e3, 3)
                grid_of = collections.Counter(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) for r in sel)
                loop_grid[name] = grid_of.most_common(1)[0][0]  # the PMC pass is matched on it
        for name, fn, head in (
                ("k_copy_rows", "gather_launches", "# (512*256, 5) = learner gather (rth_replay_gather, B=512, 5 columns)"),
                (CONV2, "conv2_launches", "# learner stream = the learner's [s0; s1] forward (2B = 1024 samples; "
                                          "bench.py's live roofline_conv2); the actor stream: target pass (512), actors (256)"),
                (CONV3, "conv3_launches", "# learner stream = the learner's [s0; s1] forward (2B = 1024 samples; "
                                          "bench.py's live roofline); the actor stream: target pass (512), actors (256)")):
            by_grid = collections.defaultdict(list)
            for r in win:
                if (is_conv(name, r["Kernel_Name"]) if isinstance(name, tuple) else name in r["Kernel_Name"]):
                    where = "learner stream" if r.get("Stream_Id") == learner_stream else f"stream {r.get('Stream_Id')}"
                    by_grid[(r["Grid_Size_X"], r["Grid_Size_Y"], where)].append(
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            with open(os.path.join(PROF, f"{tag}_{fn}.txt"), "w") as f:
                f.write(f"# {' | '.join(name) if isinstance(name, tuple) else name} launches in the timed window, "
                        f"by grid (threads x, y)\n{head}\n")
                for k, v in sorted(by_grid.items(), key=lambda kv: (int(kv[0][0]) * int(kv[0][1]), kv[0][2])):
                    f.write(f"grid={k} launches={len(v)} avg_us={st.mean(v) / 1e3:.2f} min_us={min(v) / 1e3:.2f} "
                            f"max_us={max(v) / 1e3:.2f}\n")
    pf = os.path.join(OUT, "pmc_fetch", "run_counter_collection.csv")
    pw = os.path.join(OUT, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(pf) and os.path.exists(pw):
        def load(p, name):
            """(kernel, grid) -> counter values in dispatch order (the two passes run the same
            command, so the k-th dispatch of a class in one is the k-th in the other)"""
            d = collections.defaultdict(list)
            rows = [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == name]
            rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
            for r in rows:
                d[(r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
            return d

        fe, wr = load(pf, "FETCH_SIZE"), load(pw, "WRITE_SIZE")
        with open(os.path.join(PROF, f"{tag}_pmc.txt"), "w") as f:
            f.write("# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB per dispatch (median)\n")
            f.write("# hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (gfx950: FETCH_SIZE counts half)\n")
            for k in sorted(set(fe) | set(wr)):
                fv, wv = st.median(fe.get(k, [0])), st.median(wr.get(k, [0]))
                f.write(f"{k[0]:24s} grid={k[1]:>9d} n={len(fe.get(k, [])):4d} FETCH_KiB={fv:12.1f} "
                        f"WRITE_KiB={wv:12.1f} hbm_MB={(2 * fv + wv) * 1024 / 1e6:10.2f}\n")
        out = {"correction": "hbm bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 half-counts FETCH_SIZE "
                             "on wide coalesced reads), median over the dispatches of each pass",
               "passes": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs of bench.py",
               # bench.py traffic_signature of the profiled command: bench quotes these bytes only
               # in a line whose own run has the same signature (defaults = the default command)
               "measured_on": {"world": arg("--world", 1), "num_actions": arg("--actions", 6),
                               "batch_size": arg("--batch", 512), "n_actors": arg("--actors", 256),
                               "capacity": arg("--capacity", 1_000_000), "frame_store": bool(arg("--frame-store", 1)),
                               "frame_ids": bool(arg("--frame-ids", 1)), "env": "synthetic",
                               "actor_steps_per_update": arg("--actor-steps", 1)}}
        key = ("rth::k_copy_rows", LEARNER_GATHER_GRID)
        if key in fe and key in wr:
            out.update({"gather_kernel": "rth::k_copy_rows (learner gather, B=512, 5 columns)",
                        "gather_hbm_bytes_per_launch": round((2 * st.median(fe[key]) + st.median(wr[key])) * 1024),
                        "gather_dispatches": len(fe[key])})
        n2 = 2 * arg("--batch", 512)  # the learner's [s0; s1] forward
        for name, conv in (("conv2", CONV2), ("conv3", CONV3)):
            # the learner launch = the dispatches whose WRITE_SIZE is 2B samples' output (the
            # target pass writes B, the actors ~N: all three share the grid)
            sel, classes = [], collections.Counter()
            for k in [k for k in fe if is_conv(conv, k[0]) and k in wr]:
                for fv, wv in zip(fe[k], wr[k]):
                    samples = round(wv * 1024 / CONV_OUT_BYTES[name])
                    classes[samples] += 1
                    if samples == n2:
                        sel.append((k, fv, wv))
            if sel:
                fm, wm = st.median(v[1] for v in sel), st.median(v[2] for v in sel)
                out.update({f"{name}_kernel": sel[0][0][0] + f" (the learner's [s0; s1] forward: the dispatches "
                                                             f"writing {n2} samples' output)",
                            f"{name}_learner_hbm_bytes_per_launch": round((2 * fm + wm) * 1024),
                            f"{name}_dispatches": len(sel),
                            f"{name}_dispatches_by_samples": dict(sorted(classes.items()))})
        hbm = {}
        for name, (match, g) in HBM_KERNELS.items():
            want = loop_grid.get(name, grids.get(g))
            cs = [k for k in fe if match in k[0] and k in wr and (want is None or k[1] == want)]
            if len(cs) > 1:  # no trace to say which grid the loop launches: the most dispatched one
                cs = [max(cs, key=lambda k: len(fe[k]))]
            if len(cs) == 1:
                k = cs[0]
                hbm[name] = round((2 * st.median(fe[k]) + st.median(wr[k])) * 1024)
        if "k_adam" in hbm and "k_grad_sqsum" in hbm:  # rth_clip_adam = both launches (bench.py roofline_hbm)
            hbm["rth_clip_adam (k_grad_sqsum + k_adam)"] = hbm["k_adam"] + hbm["k_grad_sqsum"]
        if "k_adam" in hbm:  # one rank: rth_adam_prenormed = k_adam alone (the norm in the backward)
            hbm["rth_adam_prenormed (k_adam)"] = hbm["k_adam"]
        out["hbm_bytes_per_launch"] = hbm
    if inloop or os.path.exists(pf):
        if not (os.path.exists(pf) and os.path.exists(pw)):
            out = {}
            old = os.path.join(PROF, f"traffic_{tag}.json")
            if os.path.exists(old):
                out = json.load(open(old))
        if inloop:
            out["inloop_us"] = inloop
            out["inloop_source"] = "rocprofv3 --kernel-trace of bench.py (gpurun_out/prof), mean over the timed window"
        with open(os.path.join(PROF, f"traffic_{tag}.json"), "w") as f:
            json.dump(out, f, indent=1)
    print("wrote", sorted(os.listdir(PROF)))


if __name__ == "__main__":
    main()
