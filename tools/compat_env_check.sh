mkdir -p gpurun_out
U=$(timeout -k 5 120 python -c "from k8s_gpu_scheduler_amd import _native; print(_native.hip().query_all()[0]['rocr_uuid'])")
echo "uuid=$U"
for v in "CUDA_VISIBLE_DEVICES=$U" "CUDA_VISIBLE_DEVICES=0" "HIP_VISIBLE_DEVICES=$U" "HSA_CU_MASK=0:0xffffffff" "HSA_CU_MASK=0:0-31"; do
  echo "== $v"
  env ROCR_VISIBLE_DEVICES=$U $v timeout -k 5 120 python -m k8s_gpu_scheduler_amd.agent.container_probe | cut -c1-400
done
