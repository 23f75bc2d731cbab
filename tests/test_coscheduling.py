"""Permit / waiting pods (upstream framework WaitOnPermit semantics) and the Coscheduling
(gang) plugin: a multi-pod GPU job binds all-or-nothing."""
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import parse_config
from k8s_gpu_scheduler_amd.framework.interface import Code, Status
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger

PROFILE = {
    "apiVersion": "kubescheduler.config.k8s.io/v1beta3",
    "kind": "KubeSchedulerConfiguration",
    "profiles": [{
        "schedulerName": C.SCHEDULER_NAME,
        "plugins": {
            "preFilter": {"enabled": [{"name": "GPU"}, {"name": "Coscheduling"}]},
            "filter": {"enabled": [{"name": "GPU"}]},
            "postFilter": {"enabled": [{"name": "Coscheduling"}]},
            "preScore": {"enabled": [{"name": "GPU"}]},
            "score": {"enabled": [{"name": "GPU", "weight": 10100}]},
            "reserve": {"enabled": [{"name": "GPU"}, {"name": "Coscheduling"}]},
            "permit": {"enabled": [{"name": "Coscheduling"}]},
            "preBind": {"enabled": [{"name": "GPU"}]},
        },
        "pluginConfig": [{"name": "Coscheduling", "args": {"permitWaitingTimeSeconds": 30}}],
    }],
}


def _world(nodes=2):
    fc = FakeCluster()
    for i in range(nodes):
        fc.create("nodes", O.make_node(f"n{i}", gpus=8))
    ledger = DeviceLedger()
    s = Scheduler(fc, parse_config(PROFILE), full_registry(), bind_async=False, seed=0, extras={"ledger": ledger})
    s.start_informers()
    return fc, s, ledger


def _member(name, group, size, gpus):
    return O.make_pod(name, gpus=gpus, labels_={"scheduling.x-k8s.io/pod-group": group},
                      annotations_={"pod-group.scheduling.sigs.k8s.io/min-available": str(size)})


def _bound(fc):
    return {O.name(p): O.node_name_of(p) for p in fc.list("pods")[0] if O.node_name_of(p)}


def test_gang_binds_only_when_complete():
    fc, s, ledger = _world()
    fc.create("pods", _member("job-0", "job", 3, 4))
    fc.create("pods", _member("job-1", "job", 3, 4))
    r = s.schedule_pending()
    assert all(not x.status.ok for x in r)          # 2 of 3 members: not even tried
    assert _bound(fc) == {} and not s.waiting_pods()
    fc.create("pods", _member("job-2", "job", 3, 4))
    s.queue.move_all_to_active_or_backoff()
    s.queue.initial_backoff_s = 0.0
    import time
    time.sleep(0.01)
    for _ in range(5):
        s.schedule_pending()
        if len(_bound(fc)) == 3:
            break
        time.sleep(1.05)                           # members still in their first backoff
    b = _bound(fc)
    assert sorted(b) == ["job-0", "job-1", "job-2"] and not s.waiting_pods()
    # 3 x 4 GPUs on 2 x 8: every member got a xGMI quad, ledger holds 12 GPUs
    assert sum(1 for n in ("n0", "n1") for st in ledger.devices(n) if st.pods) == 12


def test_members_wait_at_permit_then_release_together():
    fc, s, ledger = _world()
    for i in range(3):
        fc.create("pods", _member(f"g-{i}", "g", 3, 4))
    first = s.schedule_pending(max_pods=2)
    assert [x.status.code for x in first] == [Code.WAIT, Code.WAIT]
    assert set(s.waiting_pods()) == {"default/g-0", "default/g-1"} and _bound(fc) == {}
    assert sum(1 for n in ("n0", "n1") for st in ledger.devices(n) if st.pods) == 8   # reserved, not bound
    (last,) = s.schedule_pending()
    assert last.status.ok and len(_bound(fc)) == 3 and not s.waiting_pods()


def test_gang_that_cannot_fit_releases_its_reservations():
    fc, s, ledger = _world()
    for i in range(3):                               # 3 x 8 GPUs on 2 nodes: cannot all fit
        fc.create("pods", _member(f"big-{i}", "big", 3, 8))
    res = s.schedule_pending()
    assert _bound(fc) == {} and not s.waiting_pods()
    assert all(not st.pods for n in ("n0", "n1") for st in ledger.devices(n))
    assert any("rejected at permit" in " ".join(x.status.reasons) for x in s.results)
    assert any(x.status.code == Code.UNSCHEDULABLE for x in res)


def test_waiting_pod_times_out():
    fc, s, ledger = _world()
    for i in range(2):
        fc.create("pods", _member(f"t-{i}", "t", 2, 1))
    cos = s.frameworks[C.SCHEDULER_NAME].plugin("Coscheduling")
    cos.timeout_s = 0.0                              # expire at once
    (r0,) = s.schedule_pending(max_pods=1)
    assert r0.status.code == Code.WAIT
    assert s.expire_waiting() == 1 and not s.waiting_pods()
    assert all(not st.pods for n in ("n0", "n1") for st in ledger.devices(n))


def test_handle_allow_and_reject_api():
    fc, s, _ = _world()
    for i in range(2):
        fc.create("pods", _member(f"h-{i}", "h", 2, 1))
    (r0,) = s.schedule_pending(max_pods=1)
    wp = s.handle.get_waiting_pod("default/h-0")
    assert wp is not None and wp.pending == {"Coscheduling"} and wp.node
    assert s.handle.allow("default/h-0", "Coscheduling")
    assert _bound(fc) == {"h-0": wp.node} and s.handle.get_waiting_pod("default/h-0") is None
    assert not s.handle.reject("default/h-0", "x", "gone")      # not waiting any more
    assert Status.wait("m").code == Code.WAIT
