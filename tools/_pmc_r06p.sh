cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in -1 4 2; do
  T8_VARIANT=$v timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/r06p_t8_v$v -o run -- python3 tools/pmc_table8.py > $OUT/r06p_t8_v$v.log 2>&1 || exit 3
  python3 tools/pmc_table8.py --reduce $OUT/r06p_t8_v$v/run_counter_collection.csv $OUT/r06p_t8_v$v.json > $OUT/r06p_t8_v${v}_reduce.log 2>&1
done
SAMPLE_VARIANTS=8,23,26,28,29 timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/r06p_sample -o run -- python3 tools/pmc_sample.py > $OUT/r06p_sample.log 2>&1 || exit 4
python3 tools/pmc_sample.py --reduce $OUT/r06p_sample/run_counter_collection.csv $OUT/r06p_sample.json > $OUT/r06p_sample_reduce.log 2>&1
KB_SEEDED_ONLY=1 KB_SEEDED_VARIANTS=0,8,23,26,28,29,30 timeout -k 10 300 python3 tools/kbench_sample.py > $OUT/r06p_kbench_sample.log 2>&1
