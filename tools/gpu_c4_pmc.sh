cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/c4pmc
mkdir -p $O
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g -d $O/p$i -o run --output-format csv -- python tools/bench_configs.py c4 --steps 3 --warmup 2 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/p$i.log; [ $rc -ge 124 ] && exit $rc; }
done
python tools/pmc_summary.py $O 2>&1 | grep -E "k_radix_scatter|k_scan_emit_x|k_render_fwd|k_radix_hist|k_preprocess" | cut -c1-400
