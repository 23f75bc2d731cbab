mkdir -p gpurun_out
for r in 1 2; do for m in base pod4 pod5 pod4s pod5s; do
  SKIP_CURVE=1 SPLIT_KS=4,5 MODES=$m timeout -k 10 120 python -u tools/phase_split_study.py > gpurun_out/ps_$m_$r.log 2>&1 || exit 1
  echo "$r $m $(tail -1 gpurun_out/ps_$m_$r.log)"
done; done
