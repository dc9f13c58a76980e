set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_attn
mkdir -p $O
python -u $R/tools/attn_one.py 32 1500 40 > $O/time.txt
python -u $R/tools/attn_one.py 1 1500 40 >> $O/time.txt
for shape in "1 1500" "32 1500"; do
  tag=$(echo $shape | tr ' ' _)
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1_$tag -o p -- python $R/tools/attn_one.py $shape 10 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p2_$tag -o p -- python $R/tools/attn_one.py $shape 10 > /dev/null
done
