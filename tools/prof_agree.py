"""Checks that rocprofv3's per-launch kernel durations agree with bench.py's own HIP-event
timing of the headline kernel, phase by phase (the kernel-stats CSV averages every launch
of a kernel name, including bench's n = 1 host-boundary calls, so its overall mean is not
the headline's).

Usage: python tools/prof_agree.py <run_kernel_trace.csv> <bench_line.json> [out.json]
"""
import csv
import json
import statistics
import sys

KERNEL = "void hg::solve_aos<0, true, float, 2, 39>"


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(KERNEL)]
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    line = json.load(open(sys.argv[2]))
    warm, steps = line["warmup"], line["steps"]
    stats_n = line["launch_stats"]["launches"]
    ref_loops = line["reference_statistic"]["loops"]
    a = warm
    timed = us[a:a + steps]
    a += steps
    per = us[a:a + stats_n]
    a += stats_n + 1  # reference_statistic's one calibration launch
    ref = us[a:a + ref_loops]
    out = {
        "kernel": KERNEL,
        "launches_in_trace": len(us),
        "timed_steps": {"rocprof_mean_us": round(statistics.mean(timed), 2),
                        "bench_launch_us": round(line["roofline"]["launch_ms"] * 1e3, 2)},
        "launch_stats": {"rocprof_median_us": round(statistics.median(per), 2),
                         "bench_median_us": line["launch_stats"]["median_us"],
                         "bench_samples": "means of groups of back-to-back launches"},
        "reference_statistic": {"rocprof_mean_us": round(statistics.mean(ref), 2),
                                "bench_mean_us": line["reference_statistic"]["mean_us"],
                                "loops": ref_loops},
    }
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
