#!/usr/bin/env bash
# One GPU-box session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash / abort / timeout ends the script
# (a plain test failure, exit 1, does not).  Usage (from the repo root):
#   gpurun -- bash tools/gpu_round.sh [tag] [steps...]
set -u
TAG="${1:-r01}"
shift || true
STEPS="${*:-smoke tests bench prof}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() {  # exit codes that mean the GPU run did not end normally
    case "$1" in 0|1|2|3|4|5) return 1 ;; *) return 0 ;; esac
}

run() {  # run <name> <seconds> <cmd...>
    local name="$1" secs="$2"; shift 2
    echo "=== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -n 5 "$OUT/$name.log"
    if [ "$rc" != 0 ]; then  # every failed step's whole log is kept (a later step may reuse the name)
        mkdir -p "$OUT/failed"
        cp "$OUT/$name.log" "$OUT/failed/${TAG}_${name}_rc${rc}_$(date +%H%M%S).log"
    fi
    if fatal "$rc"; then echo "FATAL rc=$rc in $name: stopping"; exit "$rc"; fi
    return 0
}

rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
# device memory already in use before any step of ours (another process on the card shows here)
rocm-smi --showmeminfo vram >> "$OUT/rocm_smi.txt" 2>&1 || true
lscpu > "$OUT/lscpu.txt" 2>&1 || true
for step in $STEPS; do
    case "$step" in
        smoke) run smoke 300 python __graft_entry__.py smoke ;;
        lasterror) run lasterror 60 tools/_build/probe_lasterror ;;
        cpuprobe) run cpuprobe 60 bash tools/cpu_probe.sh ;;
        crossover) run crossover 400 python tools/crossover.py ;;
        chunk_probe) run chunk_probe 300 python tools/chunk_probe.py ;;
        kbench_gpt) run kbench_gpt 300 python tools/kbench_gpt.py ;;
        ransac_tests) run pytest_ransac 600 python -u -m pytest tests/test_gpu_ransac.py tests/test_gpu_large.py \
                -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        gpt_tests) run pytest_gpt 600 python -u -m pytest tests/test_gpu_refcu.py tests/test_gpu_parity.py \
                tests/test_gpu_grouped.py -m gpu -q -k "gpt or refcu or reference_kernels or ge" \
                -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        pmc_tlb)
            # translation-cache counters of the headline kernel at 1 GB and 2 GB (one pass, no tracing)
            run pmc_tlb 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum \
                GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_tlb_$TAG" -o run -- \
                python3 tools/pmc_tlb.py
            python3 tools/pmc_tlb.py --reduce "$OUT/pmc_tlb_$TAG/run_counter_collection.csv" \
                "$OUT/pmc_tlb_$TAG.json" > /dev/null || true ;;
        cpubase) run cpubase 300 python -c "import bench, json; print(json.dumps(bench.cpu_baseline(10_000_000)))" ;;
        newtests) run pytest_new 600 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_kat.py \
                tests/test_gpu_config5.py tests/test_gpu_host.py tests/test_gpu_cpp_api.py -m gpu -v \
                -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        vanilla_tests) run pytest_vanilla 600 python -u -m pytest tests/test_gpu_vanilla_grad.py tests/test_gpu_parity.py \
                tests/test_gpu_kat.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        rect_tests) run pytest_rect 600 python -u -m pytest tests/test_gpu_rect_grad.py tests/test_gpu_rect_bcast.py \
                tests/test_gpu_rect_aten_bits.py tests/test_gpu_offsets.py tests/test_gpu_parity.py -m gpu -v -s \
                -k "rect or offsets or grad" -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        autograd_cost) run autograd_cost 300 python -u tools/autograd_cost.py ;;
        rocm_grad_probe) run rocm_grad_probe 300 python -u tools/rocm_grad_probe.py ;;
        rocm_grad_probe2) run rocm_grad_probe2 300 python -u tools/rocm_grad_probe2.py ;;
        multi_tests) run pytest_multi 300 python -u -m pytest tests/test_gpu_multi.py tests/test_multi_capi.py -v \
                -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        gpus2_bare)
            # the driver-shaped bare command with --gpus 2 and no torchrun: bench.py starts the
            # two ranks itself (gloo: they share the one GPU here) and prints n_gpus 2
            run gpus2_bare 400 python bench.py --gpus 2 --steps 20 --warmup 2 --no-extras \
                --dist-backend gloo ;;
        prof_rect_bwd) run prof_rect_bwd 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/prof_rect_bwd_$TAG" -o run -- python3 tools/prof_rect_bwd.py ;;
        aten_tests) run pytest_aten 600 python -u -m pytest tests/test_gpu_aten_sum.py tests/test_gpu_rect_grad.py \
                tests/test_gpu_rect_bcast.py tests/test_gpu_offsets.py tests/test_gpu_vanilla_grad.py -m gpu -v \
                -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --tb=long -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        driver_tests)  # the driver's own command, verbatim
            run pytest_driver 900 python -m pytest tests/ -x -q -m gpu ;;
        tests_prof)
            # the whole GPU suite under a kernel trace: if anything faults, the trace names the
            # last kernels dispatched before it
            run pytest_prof 1100 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/tests_prof_$TAG" -o run -- python3 -u -m pytest tests -m gpu -x -v \
                -p no:cacheprovider --timeout 300 --timeout-method thread
            gzip -f "$OUT/tests_prof_$TAG"/*kernel_trace.csv 2>/dev/null || true ;;
        bench) run bench 600 python bench.py ;;
        prof)
            run prof 900 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/prof_$TAG" -o run -- python3 bench.py --no-cpu
            # the per-launch trace (~50 K launches) is reduced here and compressed, so the
            # session's output stays under gpurun's 64 MiB copy-back limit
            grep '^{' "$OUT/prof.log" > "$OUT/prof_$TAG/bench_line.json" || true
            python3 tools/prof_agree.py "$OUT/prof_$TAG/run_kernel_trace.csv" \
                "$OUT/prof_$TAG/bench_line.json" "$OUT/prof_$TAG/prof_agreement.json" > /dev/null || true
            gzip -f "$OUT/prof_$TAG/run_kernel_trace.csv" || true ;;
        pmc)
            # HBM traffic: separate passes (FETCH_SIZE and WRITE_SIZE can't share one), no
            # tracing domains; a fixed short dispatch list (tools/pmc_run.py)
            run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
                -d "$OUT/pmc_fetch_$TAG" -o run -- python3 tools/pmc_run.py
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
                -d "$OUT/pmc_write_$TAG" -o run -- python3 tools/pmc_run.py ;;
        pmc_reduce)
            # reduce the passes on the box itself (same tree, same library) so the bench that
            # follows in this call reads the fresh figures; the summary comes back in gpurun_out
            PMC_TAG="$TAG" python3 tools/pmc_traffic.py "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG" \
                profiles/pmc_traffic.json > "$OUT/pmc_reduce.log" 2>&1 \
                && cp profiles/pmc_traffic.json "$OUT/pmc_traffic_$TAG.json" ;;
        pmc_score)
            run pmc_score 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES \
                SQ_WAVE_CYCLES SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE --kernel-trace \
                --output-format csv -d "$OUT/pmc_score_$TAG" -o run -- python3 tools/pmc_score.py ;;
        pmc_sample)
            run pmc_sample 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES \
                SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
                --kernel-trace --output-format csv -d "$OUT/pmc_sample_$TAG" -o run -- \
                python3 tools/pmc_sample.py
            python3 tools/pmc_sample.py --reduce "$OUT/pmc_sample_$TAG/run_counter_collection.csv" \
                "$OUT/pmc_sample_valu.json" > "$OUT/pmc_sample_reduce.log" 2>&1 || true ;;
        pmc_table8)
            # the fused Table-8 kernel (draws + gather + solve, binary64) at 10 M, ACA then SKS:
            # VALU / SALU / LDS instructions, VALU busy, residency, waits (one pass, no tracing)
            run pmc_table8 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES \
                SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
                --kernel-trace --output-format csv -d "$OUT/pmc_table8_$TAG" -o run -- \
                python3 tools/pmc_table8.py
            python3 tools/pmc_table8.py --reduce "$OUT/pmc_table8_$TAG/run_counter_collection.csv" \
                "$OUT/pmc_table8_$TAG.json" > "$OUT/pmc_table8_reduce.log" 2>&1 || true ;;
        sample_flags) run sample_flags 200 bash tools/sample_flags_probe.sh run ;;
        slp_ab) run slp_ab 300 python tools/slp_ab.py ;;
        kbench) run kbench 600 python tools/kbench.py ;;
        kbench_soa) run kbench_soa 600 python tools/kbench_soa.py ;;
        kbench_score) run kbench_score 600 python tools/kbench_score.py ;;
        op_overhead) run op_overhead 300 python tools/op_overhead.py ;;
        kbench_rect) run kbench_rect 300 python tools/kbench_rect.py ;;
        kbench_sample) run kbench_sample 300 python tools/kbench_sample.py ;;
        kbench_seeded) KB_SEEDED_ONLY=1 run kbench_seeded 300 python tools/kbench_sample.py ;;
        kbench_pair)  # the packed-pair seeded forms against the shipped one, ACA then SKS
            KB_ROUNDS=11 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,7,8,10,11,12 run kbench_pair 300 python tools/kbench_sample.py
            KB_ROUNDS=11 KB_ALGO=1 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,7,8,10,11,12 run kbench_pair_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_pair_idx)  # the packed-pair indexed form against the shipped one, ACA then SKS
            KB_ROUNDS=11 KB_INDEXED_VARIANTS=0,2,8 KB_SEEDED_VARIANTS=0,13 run kbench_pair_idx 300 python tools/kbench_sample.py
            KB_ROUNDS=11 KB_ALGO=1 KB_INDEXED_VARIANTS=0,2,8 KB_SEEDED_VARIANTS=0,13 run kbench_pair_idx_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_pkdiv)  # packed-pair divisions (shipped) vs the round-2 scalar-division pairs, ACA then SKS
            KB_ROUNDS=11 KB_INDEXED_VARIANTS=0,8,9 KB_SEEDED_VARIANTS=0,10,12 run kbench_pkdiv 300 python tools/kbench_sample.py
            KB_ROUNDS=11 KB_ALGO=1 KB_INDEXED_VARIANTS=0,8,9 KB_SEEDED_VARIANTS=0,10,12 run kbench_pkdiv_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_gather) run kbench_gather 300 python tools/kbench_gather.py ;;
        kbench_mrg) run kbench_mrg 300 python tools/kbench_mrg.py ;;
        kbench_t8q) run kbench_t8q 300 python tools/kbench_t8q.py ;;
        kbench_mrg_words) run kbench_mrg_words 300 python tools/kbench_mrg_words.py ;;
        t8_order) run t8_order 300 python tools/t8_order_probe.py ;;
        single_call) run single_call 120 tools/_build/single_call_probe ;;
        kbench_gather_st) KB_ROUNDS=11 KB_GATHER_VARIANTS=0,7,3 run kbench_gather_st 300 python tools/kbench_gather.py ;;
        kbench_stp)  # the seeded sampler's H stores under other cache policies, ACA then SKS
            KB_ROUNDS=11 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,22,23,24,25,26,27 run kbench_stp 300 \
                python tools/kbench_sample.py
            KB_ROUNDS=11 KB_ALGO=1 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,22,23,24,25,26,27 run kbench_stp_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_ablate8)  # the 8-wave packed-pair shape (SKS shipped) without remainder / hash, SKS then ACA
            KB_ROUNDS=11 KB_ALGO=1 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,19,20,21 run kbench_ablate8_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_ablate)  # where the seeded sampler's time goes, and the binary64 remainder
            KB_ROUNDS=11 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,13,14,15,16,17 run kbench_ablate 300 python tools/kbench_sample.py
            KB_ROUNDS=11 KB_ALGO=1 KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,18 run kbench_ablate_sks 300 \
                python tools/kbench_sample.py ;;
        kbench_soa_small) run kbench_soa_small 300 python tools/kbench_soa_small.py ;;
        launch_floor) run launch_floor 300 python tools/launch_floor.py ;;
        kbench_bwd) run kbench_bwd 300 python tools/kbench_bwd.py ;;
        pin_probe)  # which host copies HIP maps in place, and what KFD keeps mapped
            AMD_LOG_LEVEL=4 run pin_probe 120 python tools/pin_probe.py
            cp "$OUT/pin_probe.json" "$OUT/pin_probe_$TAG.json" 2>/dev/null || true ;;
        hbm_ceilings) run hbm_ceilings 300 python tools/hbm_ceilings.py ;;
        kbench_f64) run kbench_f64 300 python tools/kbench_f64.py ;;
        soa_streams) run soa_streams 300 python tools/soa_streams.py ;;
        soa_streams_f64)  # the 25-row pattern at the binary64 10 M size, beside the shipped solvers
            SOA_READ_TOTAL=1280000000 SOA_SHAPES=0 SOA_SOLVE=1 run soa_streams_f64 300 python tools/soa_streams.py ;;
        hbm_policy) run hbm_policy 300 python tools/hbm_policy.py ;;
        host_probe) run host_probe 300 python tools/host_probe.py ;;
        numa_probe) run numa_probe 300 python tools/numa_probe.py ;;
        dist2)
            # rehearse the N>1 control path (barriers, max-over-ranks, one JSON line) with
            # 2 ranks sharing the one GPU over gloo; the real N>1 run uses RCCL
            run dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 \
                --warmup 2 --no-extras --dist-backend gloo ;;
        dist4)
            # four ranks over gloo on the one GPU (the split / gather with 3 peers)
            run dist4 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
                --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --steps 10 \
                --warmup 2 --no-extras --dist-backend gloo ;;
        dist2_full)
            # the driver's N>1 command as it runs it (every extra section on), 2 ranks sharing
            # the one GPU over gloo: all sections keep the ranks in step to the one JSON line
            run dist2_full 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29525 bench.py --gpus 2 --steps 20 \
                --warmup 2 --dist-backend gloo ;;
        dist2_fail)
            # the extras guard: rank 1 fails as the extras start; rank 0 must still print the
            # headline line (with extras_error) -- directly or through the extras watchdog
            run dist2_fail 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29527 bench.py --gpus 2 --steps 20 \
                --warmup 2 --dist-backend gloo --inject-extras-failure 1 --extras-deadline 60 ;;
        dist2_deadline)
            # the split / gather watchdog: a deadline too short to meet ends every rank and
            # rank 0 still prints the measured line, with the stall recorded
            run dist2_deadline 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --steps 20 \
                --warmup 2 --no-extras --dist-backend gloo --gather-deadline 0.001 ;;
        dist8_small)
            # eight gloo ranks sharing the one GPU, every section on, 1 M problems per rank: the
            # N = 8 control path end to end (NUMA records, split / gather with 7 peers, the
            # host-sharded batch allocated by 8 ranks) in a few minutes
            run dist8_small 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
                --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --steps 20 \
                --warmup 2 --problems-per-gpu 1000000 --dist-backend gloo --extras-deadline 500 ;;
        torchrun1)
            run torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 50 \
                --warmup 5 --no-extras --no-cpu ;;
        *) echo "unknown step $step" ;;
    esac
done
echo "done"
