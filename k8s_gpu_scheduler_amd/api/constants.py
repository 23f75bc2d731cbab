"""Names, keys and constants shared by every layer.

The reference hard-codes most of these inline; here they are
collected once and every former constant is overridable through the plugin args
(`framework/config.py`).

Parity citations:
  * plugin name "GPU"                      -- reference pkg/plugins/gpu_plugin/gpu_plugins.go:50
  * scheduler name "gpu-scheduler"         -- reference deploy/scheduler.yaml:15
  * Score weight 10100                     -- reference deploy/scheduler.yaml:20
  * MIG layouts all-{4g,2g,1g}             -- reference gpu_plugins.go:52
  * NodePorts 32767/32700/30090            -- reference gpu_plugins.go:185,317,363
  * Redis password "1234"                  -- reference gpu_plugins.go:363
  * MPS limits / thread percentages        -- reference gpu_plugins.go:896-903
"""

PLUGIN_NAME = "GPU"
SCHEDULER_NAME = "gpu-scheduler"
DEFAULT_SCORE_WEIGHT = 10100

MIN_NODE_SCORE = 0
MAX_NODE_SCORE = 100

# ---- MI355X hardware model ---------------------------------------------------------
MI355X = "MI355X"
MI355X_CUS = 256
MI355X_XCDS = 8
MI355X_HBM_GIB = 288
MI355X_XGMI_LINKS = 7
MI355X_XGMI_LINK_GBPS = 153.0
MI355X_BF16_DENSE_TFLOPS = 2500.0
MI355X_HBM_TBPS = 8.0

# Compute partition modes -> partitions per GPU ("<N>P" in the recommender matrices).
COMPUTE_PARTITIONS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
PARTITIONS_TO_MODE = {v: k for k, v in COMPUTE_PARTITIONS.items()}
MEMORY_PARTITIONS = {"NPS1": 1, "NPS2": 2}

# ---- Kubernetes resource names / labels / annotations -------------------------------
RESOURCE_GPU = "amd.com/gpu"              # whole GPUs (or whole partitions)
RESOURCE_GPU_CU = "amd.com/gpu-cu"        # fractional: compute units out of 256
RESOURCE_GPU_MEM = "amd.com/gpu-memory"   # fractional: HBM in GiB
RESOURCE_CPU = "cpu"
RESOURCE_MEMORY = "memory"
RESOURCE_PODS = "pods"
RESOURCE_EPHEMERAL_STORAGE = "ephemeral-storage"

LABEL_GPU_PRODUCT = "amd.com/gpu.product-name"
LABEL_GPU_COUNT = "amd.com/gpu.count"
LABEL_COMPUTE_PARTITION = "amd.com/compute-partition"
LABEL_MEMORY_PARTITION = "amd.com/memory-partition"
LABEL_MIG_CONFIG = "nvidia.com/mig.config"          # parity mode only
TAINT_PARTITIONING = "amd.com/partitioning"
# set by the node agent while a fabric / RCCL set probe runs (agent.probes)
TAINT_PROBING = "amd.com/fabric-probe"

ANNOT_PREFIX = "gpu-scheduler.amd.com/"
# upstream kube-scheduler NodePreferAvoidPods annotation (JSON AvoidPods)
ANNOT_PREFER_AVOID_PODS = "scheduler.alpha.kubernetes.io/preferAvoidPods"
ANNOT_DEVICES = ANNOT_PREFIX + "devices"            # comma separated device UUIDs
ANNOT_DEVICE_INDICES = ANNOT_PREFIX + "device-indices"
ANNOT_CU_MASK = ANNOT_PREFIX + "cu-mask"
ANNOT_SLO = ANNOT_PREFIX + "slo"
ANNOT_WORKLOAD = ANNOT_PREFIX + "workload"
ANNOT_RESIZED = ANNOT_PREFIX + "resized-request"
ANNOT_NODE_SCORE = ANNOT_PREFIX + "score"
# node annotation kept by the agent: JSON {uuid: reason} of unhealthy devices ("{}" when
# all are healthy) -- also the change trigger that makes schedulers re-read the inventory
ANNOT_UNHEALTHY = ANNOT_PREFIX + "unhealthy-devices"
# pod annotation "partition": the pod needs a hard-isolated compute partition (its own
# XCDs / HBM share) rather than a CU-mask share of a GPU; its size is its amd.com/gpu-cu
# request, or ANNOT_PARTITION_CUS as chosen by the partition controller from predictions
ANNOT_ISOLATION = ANNOT_PREFIX + "isolation"
ANNOT_PARTITION_CUS = ANNOT_PREFIX + "partition-cus"
# node annotations kept by the agent: the probed partition capabilities (JSON
# PartitionCaps) and the state of the last partition request (JSON {state, mode, ...})
ANNOT_PARTITION_CAPS = ANNOT_PREFIX + "partition-caps"
ANNOT_PARTITION_STATE = ANNOT_PREFIX + "partition-state"
# per-pod HBM overuse verdicts of the agent (node annotation, JSON {pod: {used_gib, cap_gib}})
ANNOT_HBM_OVERUSE = ANNOT_PREFIX + "hbm-overuse"

ENV_SLO = "SLO"
# batch pods: query batches the pod will run (the scheduler predicts its GPU time from it)
ENV_ITERATIONS = "ITERATIONS"
# Device env written before the container starts (PreBind) -- MI355X-native keys.
ENV_ROCR_VISIBLE = "ROCR_VISIBLE_DEVICES"
ENV_HIP_VISIBLE = "HIP_VISIBLE_DEVICES"
ENV_CU_MASK = "HSA_CU_MASK"
ENV_HBM_LIMIT = "GPU_SCHED_HBM_LIMIT_GIB"
# Reference keys kept for --compat-env (reference gpu_plugins.go:915-917).
ENV_CUDA_VISIBLE = "CUDA_VISIBLE_DEVICES"
ENV_MPS_MEM = "CUDA_MPS_PINNED_DEVICE_MEM_LIMIT"
ENV_MPS_THREADS = "CUDA_MPS_ACTIVE_THREAD_PERCENTAGE"

# ---- Service discovery (reference utils/utils.go:24-70) ----------------------------
REDIS_NODEPORT = 32767
REDIS_PASSWORD = "1234"
REDIS_NAMESPACE = "redis"
REDIS_POD_SUBSTR = "-0"
RECOMMENDER_NODEPORT = 32700
RECOMMENDER_PORT = 50051
RECOMMENDER_NAMESPACE = "recommender"
RECOMMENDER_POD_SUBSTR = "recommender"
PROMETHEUS_NODEPORT = 30090
PROMETHEUS_NAMESPACE = "prometheus"
PROMETHEUS_POD_SUBSTR = "prometheus-0"
PROFILER_POD_SUBSTR = "profiler"
EXPORTER_POD_SUBSTR = "dcgm"          # reference utils/utils.go:88 ; ours: "amd-gpu-exporter"

# ---- Reference GPU-sharing constants (parity) --------------------------------------
MIG_CONFIGS = ["all-4g.24gb", "all-2g.12gb", "all-1g.6gb"]
MPS_LIMITS = {"2": ("0=16350MB", "50"), "4": ("0=8175MB", "25")}

# Timings (reference §6.4)
INFORMER_RESYNC_S = 3.0
PROM_TIMEOUT_S = 1.0
PROFILER_POLL_S = 2.0
RECONFIGURE_POLL_S = 2.0
RECOMMENDER_JOB_DELAY_S = 30
RECOMMENDER_WORKERS = 10

DCGM_METRICS = [
    "DCGM_FI_PROF_GR_ENGINE_ACTIVE",
    "DCGM_FI_DEV_MEM_COPY_UTIL",
    "DCGM_FI_DEV_GPU_TEMP",
    "DCGM_FI_DEV_FB_USED",
    "DCGM_FI_DEV_FB_FREE",
]
# AMD exporter series (ours) -- the DCGM names above map onto these.
AMD_METRICS = [
    "amd_gpu_gfx_activity",
    "amd_gpu_umc_activity",
    "amd_gpu_temperature_hotspot",
    "amd_gpu_vram_used_mb",
    "amd_gpu_vram_free_mb",
    "amd_gpu_power_watts",
    "amd_gpu_xgmi_tx_bytes",
    "amd_gpu_xgmi_rx_bytes",
]
DCGM_TO_AMD = dict(zip(DCGM_METRICS, AMD_METRICS[:5]))
