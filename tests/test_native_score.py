"""Native node scoring (`_core.NodePack.score`, native/core/score.cpp) against the Python
Score path of the GPU plugin (`GPUPlugin._score_cands` with native_score off): the same
device and a bit-identical score on random ledgers -- residents with SLOs and interference
rows, live telemetry samples, the balance and complementarity terms, spread packing."""
import random

import pytest

from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.interface import CycleState
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.models import workloads as W
from k8s_gpu_scheduler_amd.parallel.podbench import analytic_predictions
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger
from k8s_gpu_scheduler_amd.telemetry.cache import DeviceSample, TelemetryCache

pytestmark = pytest.mark.skipif(_native.core() is None or not hasattr(_native.core(), "NodePack"),
                                reason="native core not built")


def _world(args, seed):
    fc = FakeCluster()
    for i in range(6):
        fc.create("nodes", O.make_node(f"n{i}", gpus=8))
    tele = TelemetryCache(stale_s=0)
    extras = {"ledger": DeviceLedger(), "telemetry": tele, "predictions": analytic_predictions(),
              "roofline": W.roofline_split}
    s = Scheduler(fc, default_gpu_config(args), full_registry(), bind_async=False, record_events=False, seed=seed,
                  extras=extras)
    s.start_informers()
    return fc, s, tele


@pytest.mark.parametrize("args", [
    {"w_balance": 1.0},
    {"w_balance": 1.0, "w_complement": 2.0, "w_telemetry": 0.7},
    {"w_slo": 0.0, "pack": "spread", "w_telemetry": 0.0},
    {"w_balance": 0.0, "w_pack": 0.0},
])
def test_native_node_score_matches_python(args):
    rng = random.Random(hash(str(args)) & 0xFFFF)
    fc, s, tele = _world(args, seed=1)
    gpu = s.frameworks[C.SCHEDULER_NAME].plugin("GPU")
    # populate: residents of random workloads / sizes / SLOs through the real cycle
    for i in range(90):
        wl = rng.choice(W.NAMES).replace("_", "-")
        fc.create("pods", O.make_pod(f"{wl}-r{i}", gpu_cu=rng.choice([32, 64, 128]), gpu_mem_gib=rng.choice([1, 4, 16]),
                                     slo=rng.uniform(1, 60), env={C.ENV_ITERATIONS: str(rng.randint(1, 40))}))
    s.schedule_pending()
    for nn in ("n1", "n3"):
        for st in gpu.ledger.devices(nn)[::2]:
            tele.update(nn, st.device.uuid, DeviceSample(gfx_activity=rng.random() * 1.2,
                                                          vram_used_mb=rng.uniform(0, 290) * 1024))
    checked = 0
    for i in range(60):
        wl = rng.choice(W.NAMES).replace("_", "-")
        pod = O.make_pod(f"{wl}-x{i}", gpu_cu=rng.choice([32, 64]), gpu_mem_gib=rng.choice([1, 4]),
                         slo=rng.choice([0.0, rng.uniform(1, 80)]), env={C.ENV_ITERATIONS: "10"})
        req = gpu.parse_request(pod)
        name = O.name(pod)
        conf, intf = gpu._pod_predictions(name)
        work = gpu.pod_work(pod, conf)
        for node in ("n0", "n1", "n2", "n3", "n4", "n5"):
            state = CycleState()
            cands = []
            for st in gpu.ledger.devices(node):
                if st.device.healthy and st.hbm_free + 1e-6 >= req.hbm_gib:
                    u0 = st.find_units(req.units)
                    if u0 is not None:
                        cands.append((st, u0))
            if len(cands) < 2:
                continue
            gpu.native_score = False
            py = gpu._score_cands(node, cands, req, name, conf, intf, work)
            gpu.native_score = True
            nat = gpu._score_cands(node, cands, req, name, conf, intf, work)
            assert (py is None) == (nat is None)
            if py is not None:
                assert nat.allocs == py.allocs, (node, args)
                assert nat.score == py.score, (node, nat.score, py.score)
                checked += 1
            del state
    assert checked > 50
