#!/usr/bin/env bash
# Builds the CPU checkers (test infrastructure only, never part of the product):
#   oracle/_build/libhg_oracle.so  -- our C restatement (hg_oracle.c)
#   oracle/_ref/libsks_ref.so      -- the reference's OWN ACA/SKS source, compiled
#                                     where it lies under /root/reference (skipped
#                                     when the reference is absent, e.g. on the GPU box)
#
# Numerics: -O2 -ffp-contract=off, no -march=native/-mfma.  GCC contracts a*b+c
# into FMA whenever the target has FMA, which changes ~99% of outputs bit-wise.
#
# Reference build recipe: "C++ Codes/modules/ACA_SKS.cpp" starts with
# `#include "SKS.hpp"` -- a header name that does not exist in the reference (the
# shipped header is ACA_SKS.hpp, which only pulls an unused OpenCV include).  The
# solver bodies use no symbol from either, so the recipe streams the file through
# `sed` dropping its #include line(s) and compiles it from stdin.  GE.cpp (the RHO-GE
# baseline) gets the same treatment: its only include is GE.hpp -> opencv2/core.hpp,
# and its body (OpenCV rho.cpp hFuncRefC) uses no OpenCV symbol.  No stand-in
# header is written and no reference text is copied into this repository.
#
# SKS_ORACLE_SANITIZE=<dir>: instead, build both checkers with AddressSanitizer and
# UndefinedBehaviorSanitizer into <dir> (libhg_oracle.so, libsks_ref.so; no speed build),
# for tests/test_sanitizers.py (the CPU restatement under ASan/UBSan).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REF_ROOT="${SKS_REFERENCE_ROOT:-/root/reference}"
REF_SRC="$REF_ROOT/C++ Codes/modules/ACA_SKS.cpp"
REF_GE="$REF_ROOT/C++ Codes/modules/GE.cpp"   # RHO-GE baseline (includes only GE.hpp -> OpenCV)
# The reference's GPU kernels (cal_Homo_ACA/SKS/GPT/GE) are lines 81-507 of its CUDA harness;
# the rest of that file needs OpenCV, cuRAND and nvcc's host toolchain and is not compiled.
REF_CU="$REF_ROOT/C++ Codes/Runtime Test/GPU_Runtime Test/GPU_Runtime Test.cu"
REF_CU_LINES="81,507p"
CFLAGS=(-O2 -fPIC -ffp-contract=off -fno-fast-math)
OUT_BUILD="$HERE/_build"
OUT_REF="$HERE/_ref"
SAN="${SKS_ORACLE_SANITIZE:-}"
if [[ -n "$SAN" ]]; then
    CFLAGS=(-O1 -g -fPIC -ffp-contract=off -fno-fast-math -fno-omit-frame-pointer
            -fsanitize=address,undefined -fno-sanitize-recover=all)
    OUT_BUILD="$SAN"
    OUT_REF="$SAN"
fi

mkdir -p "$OUT_BUILD"
gcc -std=c11 -D_POSIX_C_SOURCE=200809L "${CFLAGS[@]}" -shared -o "$OUT_BUILD/libhg_oracle.so" \
    "$HERE/hg_oracle.c" -lm -lpthread

if [[ -f "$REF_SRC" ]]; then
    mkdir -p "$OUT_REF"
    sed '/^[[:space:]]*#[[:space:]]*include/d' "$REF_SRC" |
        g++ -std=c++17 "${CFLAGS[@]}" -x c++ -c - -o "$OUT_REF/aca_sks_ref.o"
    sed '/^[[:space:]]*#[[:space:]]*include/d' "$REF_GE" |
        g++ -std=c++17 "${CFLAGS[@]}" -x c++ -c - -o "$OUT_REF/ge_ref.o"
    g++ -std=c++17 "${CFLAGS[@]}" -c "$HERE/ref_batch.cpp" -o "$OUT_REF/ref_batch.o"
    g++ "${CFLAGS[@]}" -shared -o "$OUT_REF/libsks_ref.so" "$OUT_REF/aca_sks_ref.o" \
        "$OUT_REF/ge_ref.o" "$OUT_REF/ref_batch.o" -lpthread
    rm -f "$OUT_REF/"*.o
    echo "built $OUT_REF/libsks_ref.so from $REF_SRC"
    if [[ -n "$SAN" ]]; then
        echo "built sanitized checkers in $SAN"
        exit 0
    fi
    # The same sources built for speed, for bench.py's CPU baseline only (never a checker):
    # -O3, AVX-512 (x86-64-v4, which the GPU boxes' EPYC 9575F has; bench checks the CPU
    # flags before loading it), FMA contraction on, LTO so the batch loop can inline the
    # solver.  Not bit-exact (about a third of the outputs keep every bit).
    NFLAGS=(-O3 -fPIC -march=x86-64-v4 -ffp-contract=fast -flto)
    sed '/^[[:space:]]*#[[:space:]]*include/d' "$REF_SRC" |
        g++ -std=c++17 "${NFLAGS[@]}" -x c++ -c - -o "$HERE/_ref/aca_sks_native.o"
    sed '/^[[:space:]]*#[[:space:]]*include/d' "$REF_GE" |
        g++ -std=c++17 "${NFLAGS[@]}" -x c++ -c - -o "$HERE/_ref/ge_native.o"
    g++ -std=c++17 "${NFLAGS[@]}" -c "$HERE/ref_batch.cpp" -o "$HERE/_ref/ref_batch_native.o"
    g++ "${NFLAGS[@]}" -shared -o "$HERE/_ref/libsks_ref_native.so" "$HERE/_ref/aca_sks_native.o" \
        "$HERE/_ref/ge_native.o" "$HERE/_ref/ref_batch_native.o" -lpthread
    rm -f "$HERE/_ref/"*.o
    echo "built oracle/_ref/libsks_ref_native.so (speed build, not bit-exact)"
fi

# A STAND-IN build of the reference's CUDA kernel statements (nvcc and the CUDA headers are
# absent: hipcc and a prepended HIP header stand in for them, so this is a cross-check of
# statement-order IEEE evaluation, not the reference's own build), compiled for gfx950 straight from the file
# (sed picks the kernel lines, oracle/ref_cu_driver.hip follows them in the same
# translation unit and launches them as the reference's host code does).  -ffp-contract=off:
# the reference's statements evaluated in order, every operation rounded on its own --
# the convention of the C++ checker above.  Needs only hipcc; runs on the GPU box.
if [[ -f "$REF_CU" && -z "$SAN" ]] && command -v hipcc > /dev/null; then
    mkdir -p "$OUT_REF"
    HIPCC="$(command -v hipcc)"
    # the kernel section must still start and end where this recipe expects
    if sed -n '81p' "$REF_CU" | grep -q '__global__ void cal_Homo_ACA' &&
       sed -n '359p' "$REF_CU" | grep -q '__global__ void cal_Homo_GE' &&
       sed -n '509p' "$REF_CU" | grep -q 'PYTHAG'; then
        # one translation unit, assembled in a scratch file outside the repository:
        # the HIP runtime header, the reference's kernel lines as they are, the driver
        TU="$(mktemp -d)/refcu.hip"
        { echo '#include <hip/hip_runtime.h>'; echo "#line 81 \"$REF_CU\"";
          sed -n "$REF_CU_LINES" "$REF_CU"; echo '#line 1 "ref_cu_driver.hip"';
          cat "$HERE/ref_cu_driver.hip"; } > "$TU"
        "$HIPCC" --offload-arch="${SKS_AMD_ARCH:-gfx950}" -O2 -fPIC -shared -ffp-contract=off \
            -fno-fast-math "$TU" -o "$OUT_REF/libsks_ref_cu.so"
        rm -rf "$(dirname "$TU")"
        echo "built oracle/_ref/libsks_ref_cu.so from $REF_CU (lines ${REF_CU_LINES%p})"
    else
        echo "reference CUDA file changed shape: oracle/_ref/libsks_ref_cu.so not built"
    fi
else
    echo "reference source absent; oracle/_ref not rebuilt"
fi
echo "built $OUT_BUILD/libhg_oracle.so"
