"""GPU health (failure detection / elastic recovery): the agent turns
amd-smi samples into per-device verdicts (agent/health.py), republishes the inventory with
`healthy` and annotates the node; the scheduler stops allocating unhealthy devices, and with
eviction on, pods on a failed GPU are deleted so their controllers reschedule them."""
import json

from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
from k8s_gpu_scheduler_amd.agent.health import HealthMonitor
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.store import schema
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
from k8s_gpu_scheduler_amd.store.resp import Redis


def _samples(n, ue=None, temp=None, dead=()):
    out = []
    for i in range(n):
        if i in dead:
            out.append({"index": i, "gfx_activity": -1, "vram_used_mb": -1, "responsive": False})
            continue
        out.append({"index": i, "gfx_activity": 10.0, "vram_used_mb": 100.0, "responsive": True,
                    "ecc_uncorrectable": float((ue or {}).get(i, 0)), "temp_c": float((temp or {}).get(i, 60))})
    return out


def _devs(n):
    return [{"uuid": f"GPU-{i}", "gpu": i} for i in range(n)]


def test_health_monitor_verdicts_and_recovery():
    hm = HealthMonitor(temp_crit_c=100, temp_hyst_c=10, miss_max=2)
    assert not hm.update(_samples(4), _devs(4))              # baseline, all healthy
    assert hm.update(_samples(4, ue={1: 3}), _devs(4))       # ECC grew on GPU 1
    assert hm.unhealthy() == {"GPU-1": "uncorrectable ECC errors"}
    assert not hm.update(_samples(4, ue={1: 3}), _devs(4))   # sticky, no transition
    assert hm.update(_samples(4, ue={1: 3}, temp={2: 101}), _devs(4))
    assert "GPU-2" in hm.unhealthy()
    assert not hm.update(_samples(4, ue={1: 3}, temp={2: 95}), _devs(4))   # inside hysteresis
    assert hm.update(_samples(4, ue={1: 3}, temp={2: 80}), _devs(4))       # recovered
    assert set(hm.unhealthy()) == {"GPU-1"}
    assert not hm.update(_samples(4, ue={1: 3}, dead=(3,)), _devs(4))      # 1 miss < miss_max
    assert hm.update(_samples(4, ue={1: 3}, dead=(3,)), _devs(4))
    assert hm.reason("GPU-3").startswith("unresponsive")
    # GPU 1 reset re-enumerates with a new UUID: the old verdict is forgotten
    devs = _devs(4)
    devs[1]["uuid"] = "GPU-1b"
    hm.update(_samples(4, ue={1: 3}), devs)
    assert hm.healthy("GPU-1b") and "GPU-1" not in hm.devices


class _Src:
    """synthetic_node with scripted samples (fault injection)."""

    def __init__(self, n):
        self.inner = synthetic_node(n, node="n1")
        self.script = _samples(n)

    def __getattr__(self, k):
        return getattr(self.inner, k)

    def samples(self):
        return list(self.script)


def _stack(evict=False, exporter=None):
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=4))
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    src = _Src(4)
    ag = NodeAgent("n1", r, src, client=fc, evict_unhealthy=evict, exporter=exporter)
    ag.step()
    s = Scheduler(fc, default_gpu_config({"pack": "spread"}), full_registry(), bind_async=False, extras={"redis": r})
    s.start_informers()
    s.queue.initial_backoff_s = 0.0           # retry at once after the node update below
    return fc, r, src, ag, s


def test_unhealthy_gpu_is_not_allocated_and_recovers():
    from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter
    ex = GpuExporter("n1")
    fc, r, src, ag, s = _stack(exporter=ex)
    src.script = _samples(4, temp={2: 120})
    ag.step()
    text = ex.render().decode()
    assert 'amd_gpu_healthy{UUID="' in text and text.count("amd_gpu_healthy{") == 4
    assert any(l.startswith("amd_gpu_healthy{") and 'gpu="2"' in l and l.endswith(" 0.0") for l in text.splitlines())
    ann = json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_UNHEALTHY])
    uuid2 = [d["uuid"] for d in schema.read_devices(r, "n1") if d["gpu"] == 2][0]
    assert list(ann) == [uuid2]
    assert [d["healthy"] for d in schema.read_devices(r, "n1")] == [True, True, False, True]
    for i in range(12):                       # 12 quarter-GPU pods: 3 healthy GPUs x 4 slots
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=64))
    res = s.schedule_pending()
    assert all(x.status.ok for x in res)
    plugin = s.frameworks[C.SCHEDULER_NAME].plugin(C.PLUGIN_NAME)
    used = {st.device.gpu for st in plugin.ledger.devices("n1") if st.pods}
    assert used == {0, 1, 3}
    fc.create("pods", O.make_pod("p-extra", gpu_cu=64))
    (extra,) = s.schedule_pending()
    assert not extra.status.ok                # the hot GPU's units are not allocatable
    src.script = _samples(4, temp={2: 50})
    ag.step()                                 # cooled down: allocatable again
    assert json.loads(O.annotations(fc.get("nodes", "n1"))[C.ANNOT_UNHEALTHY]) == {}
    res = s.schedule_pending()                # the node update moved it back to the queue
    assert res and all(x.status.ok for x in res)
    assert any(st.pods for st in plugin.ledger.devices("n1") if st.device.gpu == 2)


def test_ecc_failure_evicts_pods_when_enabled():
    fc, r, src, ag, s = _stack(evict=True)
    for i in range(4):
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=256))     # one whole-GPU share each
    assert all(x.status.ok for x in s.schedule_pending())
    victim = next(p for p in fc.list("pods")[0]
                  if O.annotations(p).get(C.ANNOT_DEVICES, "").split(",")[0] ==
                  [d["uuid"] for d in schema.read_devices(r, "n1") if d["gpu"] == 1][0])
    src.script = _samples(4, ue={1: 2})
    ag.step()
    assert ag.evicted == [O.key(victim)]
    names = {O.name(p) for p in fc.list("pods")[0]}
    assert O.name(victim) not in names and len(names) == 3


def test_synthetic_node_without_telemetry_stays_healthy():
    """A synthetic node (`agent --synthetic N`) has no telemetry source: its devices must not
    turn "unresponsive" after miss_max empty polls (they did, and a system test binding a pod
    a second after the agent started raced the flip under load)."""
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n1", gpus=0))
    r = Redis(backend=FakeRedisBackend(FakeRedisEngine()))
    ag = NodeAgent("n1", r, synthetic_node(4, node="n1"), client=fc)
    for _ in range(6):
        ag.step()
    assert ag.health.unhealthy() == {}
    assert all(d["healthy"] for d in schema.read_devices(r, "n1"))
