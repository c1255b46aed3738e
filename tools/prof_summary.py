#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/.

    python tools/prof_summary.py <tag> [--key c2_N16_B1024_polish]

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --kernel-trace --stats
summary), profiles/<tag>_summary.md (per-launch duration, HBM counters, SQ
counters) and merges the per-launch HBM traffic into profiles/pmc_traffic.json,
which bench.py reads for roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and
WRITE_SIZE are KiB per dispatch, collected in separate --pmc passes; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so the corrected
read figure is 2 x FETCH_SIZE (the engine's loads are 8-B-per-lane, for which
the guide's factor is uncalibrated -- both figures are kept).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernel="engine_kernel"):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def bench_stamp(logpath):
    """engine_src_sha of the library the profiled bench.py process loaded (its JSON line's
    "build" object), or None."""
    try:
        lines = open(logpath).read().splitlines()
    except OSError:
        return None
    for ln in reversed(lines):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            try:
                return (json.loads(ln).get("build") or {}).get("engine_src_sha")
            except ValueError:
                return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--key", default="c2_N16_B1024")
    ap.add_argument("--instances", type=int, default=1024)
    ap.add_argument("--kernel", default="engine_kernel", help="substring of the kernel the counters describe")
    ap.add_argument("--src-dir", default=None, help="the profile.sh output (default gpurun_out/prof_<tag>)")
    ap.add_argument("--out-dir", default=None, help="where the summary and pmc_traffic.json go (default profiles/)")
    a = ap.parse_args()
    src = a.src_dir or os.path.join(REPO, "gpurun_out", f"prof_{a.tag}")
    dst = a.out_dir or os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_kernel_stats.csv"))

    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    eng = [r for r in stats if a.kernel in r["Name"]]
    others = [r for r in stats if a.kernel not in r["Name"]]
    trace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
             if a.kernel in r["Kernel_Name"]]
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), a.kernel)
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"), a.kernel)
    sq = counters(os.path.join(src, "sq", "run_counter_collection.csv"), a.kernel)
    for k2, v2 in counters(os.path.join(src, "sq2", "run_counter_collection.csv"), a.kernel).items():
        if k2 != "SQ_WAVES":
            sq[k2] = v2
    f64 = counters(os.path.join(src, "f64", "run_counter_collection.csv"), a.kernel)
    # figures per solve: a sliced solve (mpcq_set_slice) is two engine launches around one
    # suspended_kernel (the compaction), both sized for the whole batch; unsliced, a solve is one
    # launch.  The counter passes replay the same launches: their kernel time is the trace's.
    grids = [int(r["Grid_Size_X"]) for r in trace]
    dispatches = len(trace) or sum(int(r["Calls"]) for r in eng)
    compactions = sum(int(r["Calls"]) for r in others if "suspended_kernel" in r["Name"])
    solves = compactions if compactions else dispatches
    solves = max(1, solves)
    kern_ms = (sum(float(r["AverageNs"]) * int(r["Calls"]) for r in eng) / solves / 1e6) if eng else None

    def mean(v):  # (per solve: the sum over its launches; one launch each when unsliced)
        return sum(v) / solves if v else None

    # every pass must have run the same build; the stamp goes into pmc_traffic.json, and
    # bench.py drops an entry whose stamp differs from the library it is running
    stamps = {p: bench_stamp(os.path.join(src, f"{p}.log")) for p in ("trace", "fetch", "write", "sq", "sq2", "f64")
              if os.path.exists(os.path.join(src, f"{p}.log"))}
    seen = {v for v in stamps.values() if v}
    if len(seen) > 1:
        raise SystemExit(f"passes of {a.tag} ran different builds: {stamps}")
    sha = seen.pop() if seen else None
    if sha is None:
        print(f"warning: no build stamp in the bench lines of {src}; the entry stays unstamped (bench.py ignores it)")

    fk, wk = mean(fetch.get("FETCH_SIZE", [])), mean(write.get("WRITE_SIZE", []))
    traffic = None
    lines = [f"# rocprofv3 summary `{a.tag}` ({a.key})", "",
             f"- build: libmpcq.so engine_src_sha `{sha}` (mpcq_build_info of the profiled process, every pass)"]
    if dispatches > solves:
        lines.append(f"- sliced solves: {dispatches} engine launches for {solves} solves (one compaction each); the "
                     f"kernel time, counters and traffic below are per solve (the sum over its launches): "
                     f"{kern_ms:.3f} ms")
    for r in eng:
        lines.append(f"- kernel `{r['Name']}`: {r['Calls']} calls, average {float(r['AverageNs']) / 1e6:.3f} ms "
                     f"(min {float(r['MinNs']) / 1e6:.3f}, max {float(r['MaxNs']) / 1e6:.3f}), "
                     f"{r['Percentage']} % of GPU time")
    for r in others:
        lines.append(f"- (other) `{r['Name'][:90]}`: {r['Calls']} calls, average {float(r['AverageNs']) / 1e3:.1f} us, "
                     f"{r['Percentage']} % of GPU time")
    if trace:
        t = trace[0]
        lines.append(f"- launch (trace fields): grid {t['Grid_Size_X']} threads, workgroup {t['Workgroup_Size_X']}, "
                     f"LDS {t['LDS_Block_Size']} B, scratch {t['Scratch_Size']} B/lane; the trace's register fields "
                     f"(VGPR_Count {t['VGPR_Count']}, Accum_VGPR_Count {t['Accum_VGPR_Count']}, SGPR_Count "
                     f"{t['SGPR_Count']}) are the dispatch's allocation fields, not the compiler's count (below)")
    # the compiler's own budget for the profiled horizon (tools/resource_usage.py)
    try:
        ru = json.load(open(os.path.join(REPO, "profiles", "resource_usage.json")))  # (the committed one)
        N = a.key.split("_N")[1].split("_")[0] if "_N" in a.key else None
        for kind, v in (ru.get(N) or {}).items():
            if kind.startswith("fused solve"):
                lines.append(f"- compiler (`-Rpass-analysis=kernel-resource-usage`, N = {N}, {kind}): VGPRs {v.get('VGPRs')}, "
                             f"AGPRs {v.get('AGPRs')}, SGPRs {v.get('TotalSGPRs')}, scratch {v.get('ScratchSize')} B/lane, "
                             f"{v.get('VGPRs Spill')} VGPRs / {v.get('SGPRs Spill')} SGPRs spilled, occupancy "
                             f"{v.get('Occupancy')} waves/SIMD, LDS {v.get('LDS Size')} B")
    except (OSError, ValueError, IndexError):
        pass
    if fk is not None and wk is not None:
        rd_raw, wr = fk * 1024, wk * 1024
        traffic = 2 * rd_raw + wr
        lines += ["", "## HBM counters (per solve)" if dispatches > solves else "## HBM counters (per launch)", "",
                  f"- FETCH_SIZE {fk:.1f} KiB -> {rd_raw / 1e6:.3f} MB raw, {2 * rd_raw / 1e6:.3f} MB with the gfx950 x2 correction",
                  f"- WRITE_SIZE {wk:.1f} KiB -> {wr / 1e6:.3f} MB",
                  f"- traffic (corrected read + write) {traffic / 1e6:.3f} MB per {'solve' if dispatches > solves else 'launch'} "
                  f"= {traffic / a.instances:.0f} B per instance"]
    if sq:
        w = mean(sq.get("SQ_WAVES", [])) or 1.0
        cyc = mean(sq.get("SQ_WAVE_CYCLES", [])) or 0.0
        lines += ["", "## SQ counters (per launch; *_CYCLES and WAIT/ACTIVE in quad-cycles)", ""]
        for name in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                     "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                     "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES"):
            v = mean(sq.get(name, []))
            if v is None:
                continue
            extra = f" ({v / w:.4g} per wave)"
            if name.startswith("SQ_WAIT") or name.startswith("SQ_ACTIVE_INST"):
                extra += f", {100 * v / cyc:.1f} % of wave cycles" if cyc else ""
            lines.append(f"- {name}: {v:.4g}{extra}")
        bc, al = mean(sq.get("SQ_LDS_BANK_CONFLICT", [])), mean(sq.get("SQ_ACTIVE_INST_LDS", []))
        if bc is not None and al:
            lines.append(f"- SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS = {bc / al:.3f} (conflict cycles per active LDS "
                         "instruction cycle)")
    fp64_flops = None
    if f64:
        fma, add, mul = (mean(f64.get(n, [])) or 0.0 for n in
                         ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64"))
        trans = mean(f64.get("SQ_INSTS_VALU_TRANS_F64", [])) or 0.0
        valu = mean(f64.get("SQ_INSTS_VALU", [])) or 0.0
        fp64_flops = (2 * fma + add + mul) * 64  # lane-ops of fully populated waves (rocprof's FP64 FLOPS formula)
        lines += ["", "## FP64 instruction counters (per launch, wave instructions)", ""]
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                     "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_MFMA_F64"):
            v = mean(f64.get(name, []))
            if v is not None:
                lines.append(f"- {name}: {v:.4g}" + (f" ({100 * v / valu:.1f} % of VALU)" if valu else ""))
        lines.append(f"- FP64 flops issued = (2 FMA + ADD + MUL) x 64 = {fp64_flops:.4g} per launch"
                     + (f" -> {fp64_flops / (kern_ms * 1e-3) / 1e12:.2f} TFLOP/s over the {kern_ms:.3f} ms launch"
                        if kern_ms else ""))
        lines.append(f"- (transcendental FP64: {trans * 64:.3g} lane-ops, not counted as flops)")
    open(os.path.join(dst, f"{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    if traffic is not None or fp64_flops is not None:
        path = os.path.join(dst, "pmc_traffic.json")
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            d = {}
        d[a.key] = {"bytes_per_launch": traffic, "fetch_kib": fk, "write_kib": wk, "tag": a.tag,
                    "engine_src_sha": sha,
                    "fp64_flops_per_launch": fp64_flops, "kernel_ms": kern_ms,
                    "launches_per_solve": dispatches / solves if solves else None,
                    "note": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section), separate --pmc passes; "
                            "fp64 flops = (2 SQ_INSTS_VALU_FMA_F64 + ADD_F64 + MUL_F64) x 64 from their own pass"}
        json.dump(d, open(path, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
