"""k8s_gpu_scheduler_amd -- an MI355X-native Kubernetes GPU scheduler.

Same capabilities as dimgatz98/k8s-gpu-scheduler (a kube-scheduler "GPU" Score/PostBind
plugin + gRPC recommender + Redis device registry + GPU profiler), re-designed for
8xMI355X nodes: scheduler framework + GPU plugin (SLO/interference, XCD-granular
fractional sharing, xGMI-aware multi-GPU placement), C++/HIP native layer (device query,
amd-smi telemetry/topology/partitions, CU-masked streams, MFMA/HBM load kernels),
RCCL-over-xGMI distributed executor and probes.  See SURVEY.md / README.md.
"""
__version__ = "0.1.0"

# compiled control-plane modules (Cython, built by _native.build) when up to date with
# their sources; pure Python otherwise or with GPUSCHED_PURE_PYTHON=1
from ._native import cyaccel as _cyaccel  # noqa: E402

_cyaccel.install()
