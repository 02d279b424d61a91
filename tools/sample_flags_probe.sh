#!/usr/bin/env bash
# Builds tools/sample_flags_probe.hip under each flag set (here, on the CPU) into
# tools/_build/sample_probe_<tag>; `run` executes them on the GPU box.
set -eu
cd "$(dirname "$0")/.."
OUT=tools/_build
if [ "${1:-build}" = build ]; then
    mkdir -p "$OUT"
    base="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -Iinclude -Isks-homography_amd/csrc"
    /opt/rocm/bin/hipcc $base tools/sample_flags_probe.hip -o "$OUT/sample_probe_default"
    /opt/rocm/bin/hipcc $base -fno-slp-vectorize tools/sample_flags_probe.hip -o "$OUT/sample_probe_noslp"
else
    for pool in synthetic tests/golden/orig_pts_wall_restated.txt; do
        for t in default noslp default noslp; do
            printf '%s %s ' "$t" "$(basename $pool)"; timeout -k 5 60 "$OUT/sample_probe_$t" "$pool"
        done
    done
fi
