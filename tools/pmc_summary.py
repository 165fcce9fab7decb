#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into committed evidence under profiles/.
usage: tools/pmc_summary.py OUTDIR TAG CONFIG [KERNEL]   (KERNEL: k_gate)

* profiles/<tag>_kernel_stats.csv  : rocprofv3 --stats output (whole run)
* profiles/<tag>_steady_state.txt  : per-kernel medians over the last 30 passes
* profiles/traffic_<cfg>.json      : the kernel's HBM bytes per launch from the
  PMC passes, calibrated (round 5, profiles/r05_fetch_calibration.txt from
  tools/ubench_fetch_cal.hip under `rocprofv3 --pmc FETCH_SIZE`, step `cal=`
  of tools/gpu_call.sh): FETCH_SIZE/WRITE_SIZE are in KiB; non-temporal
  coalesced streams of 16-B and of 8-B lanes report exactly 0.500 of the
  bytes they move, random 8-B reads from an 8-GiB table report 64 B each (one
  64-B burst per read: counted as is).  So the record stream (its algorithmic
  bytes known: 3 B per event for k_gate, 16 B for the reference-layout pass)
  is taken at 2 x its reported half, and the rest of FETCH_SIZE -- the
  gathers, the filter / bitmap / look-back traffic -- at 1x.  Round 4 doubled
  the whole FETCH_SIZE, which double-counted the gathers.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

# the kernel summarised (argv[4]; k_raw_gate for the reference-layout path)
KERNEL = sys.argv[4] if len(sys.argv) > 4 else "k_gate"


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def steady(trace_csv, n_last=30):
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a pass runs from one k_gate to the next (k_bitmap, when launched,
    # precedes the gate and is counted with the previous pass)
    idx = [i for i, r in enumerate(rows) if KERNEL in r["Kernel_Name"].split("(")[0]]
    per = {}
    starts = idx[-n_last:]
    for a in starts:
        j = a
        while j < len(rows) and (j == a or KERNEL not in rows[j]["Kernel_Name"].split("(")[0]):
            r = rows[j]
            per.setdefault(r["Kernel_Name"].split("(")[0].split("<")[0].split(" ")[-1], []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            j += 1
    spans = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
             for a, b in zip(starts[:-1], starts[1:])]
    return per, spans


def pmc_values(d, counter):
    f = find(d, "*counter_collection*.csv")
    if not f:
        return []
    vals = []
    for r in csv.DictReader(open(f)):
        if KERNEL in r.get("Kernel_Name", "").split("(")[0] and r.get("Counter_Name") == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    out, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs("profiles", exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    trace = find(os.path.join(out, "trace"), "*kernel_trace.csv")
    if stats:
        shutil.copy(stats, f"profiles/{tag}_kernel_stats.csv")
    lines = []
    if trace:
        per, spans = steady(trace)
        lines.append(f"steady state, last {len(spans) + 1} passes (us): median  min  max")
        for k, v in per.items():
            v = sorted(v)
            lines.append(f"{k:14s} {statistics.median(v):9.2f} {v[0]:9.2f} {v[-1]:9.2f}")
        if spans:
            lines.append(f"pass span median {statistics.median(spans):.2f} us")
        # the bench's timed region = the `steps` gate launches before its last
        # `steps` (the untimed sampling passes): their mean is what bench.py's
        # HIP event pair around the region measures (roofline.avg_launch_ms, which
        # also holds the dispatch gaps)
        try:
            bj = [x for x in open(os.path.join(out, "bench_trace.json")) if x.startswith("{")][-1]
            steps = json.loads(bj)["steps"]
            rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
            g = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
                 if KERNEL in r["Kernel_Name"].split("(")[0]]
            # the fused bench samples `steps` more launches after its timed ones; --raw does not
            g = g[-2 * steps:-steps] if KERNEL == "k_gate" else g[-steps:]
            lines.append(f"{KERNEL} mean over the {len(g)} timed launches {statistics.mean(g):.2f} us "
                         f"(bench HIP events, span / passes: {json.loads(bj)['roofline']['avg_launch_ms'] * 1e3:.2f} us)")
        except (OSError, IndexError, KeyError, ValueError):
            pass
    # last 10 timed k_gate launches of each PMC pass are steady state
    fetch = pmc_values(os.path.join(out, "fetch"), "FETCH_SIZE")[-10:]
    write = pmc_values(os.path.join(out, "write"), "WRITE_SIZE")[-10:]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from abnn_amd.build import kernel_source_sha

    # bench.py uses this record only while the kernel sources are these
    res = {"config": cfg, "tag": tag, "kernel": KERNEL, "source_sha": kernel_source_sha(),
           "commit": os.environ.get("ABNN_COMMIT", "")}
    if fetch and write:
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        E = 0
        try:
            bj = [x for x in open(os.path.join(out, "bench_fetch.json")) if x.startswith("{")][-1]
            c = json.loads(bj)["config"]
            E = int(c.get("visited_events_per_pass") or c.get("visited_events_per_pass_per_gpu"))
        except (OSError, IndexError, KeyError, ValueError, TypeError):
            pass
        per_event = 3 if KERNEL == "k_gate" else 16
        stream = per_event * E
        reported = f_kib * 1024
        rest = max(0.0, reported - 0.5 * stream)
        res.update({
            "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib,
            "visited_events": E,
            "stream_bytes": stream,
            "stream_bytes_formula": f"{per_event}*E (the record stream; reported by FETCH_SIZE at 0.500)",
            "other_fetch_bytes": rest,
            "other_fetch_note": "FETCH_SIZE minus the stream's reported half: the gathers (lastF / {dst, w} / "
                                "bitmap words), filter and look-back traffic, counted 1x (random 8-B reads "
                                "report one 64-B burst each)",
            "write_bytes": w_kib * 1024,
            "bytes_per_launch": stream + rest + w_kib * 1024,
            "bytes_per_launch_round4_rule": reported * 2 + w_kib * 1024,
            "correction": "calibrated: profiles/r05_fetch_calibration.txt (tools/ubench_fetch_cal.hip; "
                          "tools/gpu_call.sh cal=...): nt streams x2, the rest x1; KiB -> bytes",
            "command": "tools/profile.sh TAG c3" if KERNEL == "k_gate" else "tools/profile_raw.sh TAG",
            "launches_used": min(len(fetch), len(write)),
        })
        lines.append(f"{KERNEL} PMC per launch: FETCH_SIZE {f_kib:.0f} KiB = stream {stream/1e9:.3f} GB "
                     f"(reported at half) + other {rest/1e9:.4f} GB; WRITE_SIZE {w_kib:.0f} KiB "
                     f"({w_kib*1024/1e9:.4f} GB); total {(stream + rest + w_kib*1024)/1e9:.3f} GB "
                     f"(round-4 rule, FETCH x2: {(reported*2 + w_kib*1024)/1e9:.3f} GB)")
        with open(f"profiles/traffic_{cfg}.json", "w") as f:
            json.dump(res, f, indent=1)
    for name in ("bench_trace.json", "bench_fetch.json", "bench_write.json"):
        p = os.path.join(out, name)
        if os.path.exists(p):
            txt = open(p).read().strip().splitlines()
            if txt:
                lines.append(f"{name}: {txt[-1][:400]}")
    with open(f"profiles/{tag}_steady_state.txt", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
