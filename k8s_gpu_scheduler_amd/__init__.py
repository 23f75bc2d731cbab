"""k8s_gpu_scheduler_amd -- an MI355X-native Kubernetes GPU scheduler.

Same capabilities as dimgatz98/k8s-gpu-scheduler (a kube-scheduler "GPU" Score/PostBind
plugin + gRPC recommender + Redis device registry + GPU profiler), re-designed for
8xMI355X nodes: scheduler framework + GPU plugin (SLO/interference, XCD-granular
fractional sharing, xGMI-aware multi-GPU placement), C++/HIP native layer (device query,
amd-smi telemetry/topology/partitions, CU-masked streams, MFMA/HBM load kernels),
RCCL-over-xGMI distributed executor and probes.  See SURVEY.md / README.md.
"""
__version__ = "0.1.0"
