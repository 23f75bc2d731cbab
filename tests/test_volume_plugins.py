"""kube-scheduler volume plugins (framework/volume_plugins.py) with the fake cluster's PV
controller (kube/pv_controller.py): claim resolution, bound-volume node affinity, delayed
binding to static local volumes, dynamic provisioning with allowed topologies, zones, CSI
attach limits and disk / ReadWriteOncePod conflicts."""
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import parse_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.kube.pv_controller import PVController
from k8s_gpu_scheduler_amd.plugins import full_registry

ZONE = "topology.kubernetes.io/zone"


def _cluster(zones=("z1", "z2")):
    fc = FakeCluster()
    for i, z in enumerate(zones, 1):
        fc.create("nodes", O.make_node(f"n{i}", gpus=0, labels_={"kubernetes.io/hostname": f"n{i}", ZONE: z}))
    doc = {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": C.SCHEDULER_NAME,
                         "pluginConfig": [{"name": "VolumeBinding", "args": {"bindTimeoutSeconds": 5}}]}]}
    s = Scheduler(fc, parse_config(doc), full_registry(), bind_async=False, seed=0)
    s.start_informers()
    ctl = PVController(fc).start()
    return fc, s, ctl


def _pvc(name, size="8Gi", sc="local", modes=("ReadWriteOnce",), **spec):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"storageClassName": sc, "accessModes": list(modes), "resources": {"requests": {"storage": size}},
                     **spec}}


def _pv(name, size, sc="local", node=None, labels=None, csi=None, modes=("ReadWriteOnce",)):
    pv = {"metadata": {"name": name, "labels": dict(labels or {})},
          "spec": {"capacity": {"storage": size}, "accessModes": list(modes), "storageClassName": sc}}
    if node:
        pv["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [node]}]}]}}
    if csi:
        pv["spec"]["csi"] = csi
    return pv


def _sc(name, mode="WaitForFirstConsumer", provisioner="kubernetes.io/no-provisioner", topo=None):
    sc = {"metadata": {"name": name}, "provisioner": provisioner, "volumeBindingMode": mode}
    if topo:
        sc["allowedTopologies"] = [{"matchLabelExpressions": [{"key": ZONE, "values": list(topo)}]}]
    return sc


def _pod(name, claims=(), **spec):
    p = O.make_pod(name)
    p["spec"]["volumes"] = [{"name": c, "persistentVolumeClaim": {"claimName": c}} for c in claims]
    p["spec"].update(spec)
    return p


def _schedule(fc, s, pod):
    fc.create("pods", pod)
    (r,) = s.schedule_pending()
    return r


def test_missing_and_immediate_unbound_claims_are_unresolvable():
    fc, s, _ = _cluster()
    r = _schedule(fc, s, _pod("a", ["nope"]))
    assert not r.status.ok and 'persistentvolumeclaim "nope" not found' in r.status.message()
    fc.create("storageclasses", _sc("manual", mode="Immediate"))
    fc.create("persistentvolumeclaims", _pvc("imm", sc="manual"))          # no PV, no provisioner
    r = _schedule(fc, s, _pod("b", ["imm"]))
    assert not r.status.ok and "unbound immediate PersistentVolumeClaims" in r.status.message()


def test_bound_volume_node_affinity_pins_the_pod():
    fc, s, _ = _cluster()
    fc.create("storageclasses", _sc("manual", mode="Immediate"))
    fc.create("persistentvolumes", _pv("pv-n2", "10Gi", sc="manual", node="n2"))
    fc.create("persistentvolumeclaims", _pvc("data", sc="manual"))          # the controller binds it
    assert fc.get("persistentvolumeclaims", "data", "default")["spec"]["volumeName"] == "pv-n2"
    r = _schedule(fc, s, _pod("db", ["data"]))
    assert r.status.ok and r.node == "n2"


def test_wait_for_first_consumer_binds_the_smallest_fitting_local_volume_on_the_chosen_node():
    fc, s, _ = _cluster()
    fc.create("storageclasses", _sc("local"))
    fc.create("persistentvolumes", _pv("pv-a", "10Gi", node="n1"))
    fc.create("persistentvolumes", _pv("pv-big", "100Gi", node="n1"))
    fc.create("persistentvolumes", _pv("pv-b", "5Gi", node="n2"))
    fc.create("persistentvolumeclaims", _pvc("c1"))                         # 8Gi: only n1's volumes fit
    assert not fc.get("persistentvolumeclaims", "c1", "default")["spec"].get("volumeName")   # delayed
    r = _schedule(fc, s, _pod("p1", ["c1"]))
    assert r.status.ok and r.node == "n1"
    pvc = fc.get("persistentvolumeclaims", "c1", "default")
    assert pvc["spec"]["volumeName"] == "pv-a" and pvc["status"]["phase"] == "Bound"
    assert fc.get("persistentvolumes", "pv-a")["spec"]["claimRef"]["name"] == "c1"
    fc.create("persistentvolumeclaims", _pvc("c2", size="50Gi"))
    r = _schedule(fc, s, _pod("p2", ["c2"]))
    assert r.status.ok and r.node == "n1" and \
        fc.get("persistentvolumeclaims", "c2", "default")["spec"]["volumeName"] == "pv-big"
    fc.create("persistentvolumeclaims", _pvc("c3"))                         # nothing left that fits
    r = _schedule(fc, s, _pod("p3", ["c3"]))
    assert not r.status.ok and "didn't find available persistent volumes" in r.status.message()


def test_dynamic_provisioning_honours_allowed_topologies():
    fc, s, ctl = _cluster()
    fc.create("storageclasses", _sc("fast", provisioner="csi.example.com", topo=("z2",)))
    fc.create("persistentvolumeclaims", _pvc("scratch", sc="fast", size="20Gi"))
    r = _schedule(fc, s, _pod("job", ["scratch"]))
    assert r.status.ok and r.node == "n2" and ctl.provisioned == 1
    pvc = fc.get("persistentvolumeclaims", "scratch", "default")
    assert O.annotations(pvc)["volume.kubernetes.io/selected-node"] == "n2" and pvc["status"]["phase"] == "Bound"
    pv = fc.get("persistentvolumes", pvc["spec"]["volumeName"])
    assert pv["spec"]["nodeAffinity"]["required"]["nodeSelectorTerms"][0]["matchExpressions"][0]["values"] == ["n2"]


def test_volume_zone_of_a_bound_volume():
    fc, s, _ = _cluster()
    fc.create("storageclasses", _sc("zonal", mode="Immediate"))
    fc.create("persistentvolumes", _pv("pv-z2", "10Gi", sc="zonal", labels={ZONE: "z2__z3"}))
    fc.create("persistentvolumeclaims", _pvc("zd", sc="zonal"))
    r = _schedule(fc, s, _pod("zp", ["zd"]))
    assert r.status.ok and r.node == "n2"


def test_csi_attach_limit_per_node():
    fc, s, _ = _cluster()
    fc.create("csinodes", {"metadata": {"name": "n1"}, "spec": {"drivers": [
        {"name": "csi.example.com", "nodeID": "n1", "allocatable": {"count": 1}}]}})
    fc.create("storageclasses", _sc("csi", mode="Immediate"))
    for i in (1, 2):
        fc.create("persistentvolumes", _pv(f"vol{i}", "10Gi", sc="csi",
                                           csi={"driver": "csi.example.com", "volumeHandle": f"h{i}"}))
        fc.create("persistentvolumeclaims", _pvc(f"v{i}", sc="csi"))
    fc.create("pods", _pod("a1", ["v1"], nodeName="n1"))                    # already running on n1
    r = _schedule(fc, s, _pod("a2", ["v2"], affinity={"nodeAffinity": {
        "preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 100, "preference": {
            "matchExpressions": [{"key": "kubernetes.io/hostname", "operator": "In", "values": ["n1"]}]}}]}}))
    assert r.status.ok and r.node == "n2"        # n1 prefered but its CSI limit (1) is used


def test_disk_and_read_write_once_pod_conflicts():
    fc, s, _ = _cluster()
    disk = [{"name": "d", "gcePersistentDisk": {"pdName": "pd-1"}}]
    fc.create("pods", dict(_pod("w1", nodeName="n1"), spec=dict(_pod("w1", nodeName="n1")["spec"], volumes=disk)))
    r = _schedule(fc, s, dict(_pod("w2"), spec=dict(_pod("w2")["spec"], volumes=disk)))
    assert r.status.ok and r.node == "n2"        # pd-1 already mounted read-write on n1
    fc.create("storageclasses", _sc("rwop", mode="Immediate"))
    fc.create("persistentvolumes", _pv("solo", "10Gi", sc="rwop", modes=("ReadWriteOncePod",)))
    fc.create("persistentvolumeclaims", _pvc("one", sc="rwop", modes=("ReadWriteOncePod",)))
    assert _schedule(fc, s, _pod("u1", ["one"])).status.ok
    r = _schedule(fc, s, _pod("u2", ["one"]))
    assert not r.status.ok and "ReadWriteOncePod" in r.status.message()


def test_default_profile_enables_the_volume_plugins():
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    prof = default_gpu_config({}).profiles[0]
    assert {"VolumeBinding", "VolumeRestrictions", "VolumeZone", "NodeVolumeLimits"} <= \
        {r.name for r in prof.enabled("filter")}
    assert [r.name for r in prof.enabled("reserve")][0] == "VolumeBinding"
    assert "VolumeBinding" in [r.name for r in prof.enabled("preBind")]
