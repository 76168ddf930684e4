# PMC passes on tools/time_fields.py (fields fwd/bwd): stall/active cycles, instruction mix, LDS conflicts
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmcf1 -o run -- python $R/tools/time_fields.py > $R/gpurun_out/pmcf1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmcf2 -o run -- python $R/tools/time_fields.py > $R/gpurun_out/pmcf2.log 2>&1 || exit 1
cd $R
