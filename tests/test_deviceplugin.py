"""Kubelet device plugin (v1beta1 API over Unix sockets) against a fake kubelet: it
registers the three MI355X resources, lists devices/tokens with health and NUMA topology,
steers whole-GPU allocations to the scheduler's choice and returns each container the
assignment the scheduler recorded on its pod."""
import os
import tempfile
from concurrent import futures

import grpc

from k8s_gpu_scheduler_amd.agent import deviceplugin as dp
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger, devices_for_node


class FakeKubelet:
    def __init__(self, d):
        self.sock = os.path.join(d, "kubelet.sock")
        self.requests = []
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))

        def register(req, ctx):
            self.requests.append(req)
            return dp.Empty()
        srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(dp.REG_SERVICE, {
            "Register": grpc.unary_unary_rpc_method_handler(
                register, request_deserializer=dp.RegisterRequest.FromString,
                response_serializer=dp.Empty.SerializeToString)}),))
        srv.add_insecure_port(f"unix://{self.sock}")
        srv.start()
        self.srv = srv


def _stub(d, resource, method, req_cls, rep_cls, stream=False):
    ch = grpc.insecure_channel(f"unix://{os.path.join(d, dp.socket_name(resource))}")
    f = ch.unary_stream if stream else ch.unary_unary
    return ch, f(f"/{dp.PLUGIN_SERVICE}/{method}", request_serializer=req_cls.SerializeToString,
                 response_deserializer=rep_cls.FromString)


def _inventory(node):
    """The same inventory the scheduler derives for the node (the agent publishes one
    inventory to both)."""
    return [d.to_json() for d in devices_for_node(node)]


def test_wire_format_is_the_v1beta1_api():
    # field numbers of k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto
    r = dp.RegisterRequest(version="v1beta1", endpoint="x.sock", resource_name="amd.com/gpu")
    assert r.SerializeToString() == b"\n\x07v1beta1\x12\x06x.sock\x1a\x0bamd.com/gpu"
    c = dp.AllocateResponse()
    e = c.container_responses.add()
    e.envs["A"] = "1"
    assert c.SerializeToString() == b"\n\x08\n\x06\n\x01A\x12\x011"
    dev = dp.Device(ID="g", health="Healthy")
    assert dev.SerializeToString() == b"\n\x01g\x12\x07Healthy"


def test_register_list_health_and_allocate():
    with tempfile.TemporaryDirectory() as d:
        kubelet = FakeKubelet(d)
        fc = FakeCluster()
        fc.create("nodes", O.make_node("n1", gpus=2))
        inv = _inventory(fc.get("nodes", "n1"))
        mgr = dp.DevicePluginManager("n1", lambda: [dict(x) for x in inv], client=fc, plugin_dir=d).start()
        try:
            assert sorted(r.resource_name for r in kubelet.requests) == sorted(dp.RESOURCES)
            assert all(r.version == "v1beta1" and r.endpoint == dp.socket_name(r.resource_name)
                       for r in kubelet.requests)
            gpu_opts = [r.options for r in kubelet.requests if r.resource_name == C.RESOURCE_GPU][0]
            assert gpu_opts.get_preferred_allocation_available
            # ListAndWatch: 2 GPUs / 512 CU tokens / 576 GiB tokens; NUMA topology kept
            sizes = {}
            for res in dp.RESOURCES:
                ch, lw = _stub(d, res, "ListAndWatch", dp.Empty, dp.ListAndWatchResponse, stream=True)
                first = next(iter(lw(dp.Empty(), timeout=5)))
                sizes[res] = len(first.devices)
                assert all(x.health == "Healthy" and len(x.topology.nodes) == 1 for x in first.devices)
                ch.close()
            assert sizes == {C.RESOURCE_GPU: 2, C.RESOURCE_GPU_CU: 512, C.RESOURCE_GPU_MEM: 576}
            # health change is pushed on the open stream
            ch, lw = _stub(d, C.RESOURCE_GPU, "ListAndWatch", dp.Empty, dp.ListAndWatchResponse, stream=True)
            it = iter(lw(dp.Empty(), timeout=10))
            assert [x.health for x in next(it).devices] == ["Healthy", "Healthy"]
            inv[1]["healthy"] = False
            mgr.changed()
            assert [x.health for x in next(it).devices] == ["Healthy", "Unhealthy"]
            ch.close()
            inv[1]["healthy"] = True
            # schedule a Guaranteed 64-CU pod and a whole-GPU pod through the real framework
            s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False,
                          extras={"ledger": DeviceLedger()})
            s.start_informers()
            fc.create("pods", O.make_pod("frac", gpu_cu=64, gpu_mem_gib=16))
            fc.create("pods", O.make_pod("whole", gpus=1))
            assert all(r.status.ok for r in s.schedule_pending())
            frac, whole = fc.get("pods", "frac", "default"), fc.get("pods", "whole", "default")
            # whole GPU: kubelet asks for a preference among all GPUs -> the scheduler's choice
            ch, pref = _stub(d, C.RESOURCE_GPU, "GetPreferredAllocation", dp.PreferredAllocationRequest,
                             dp.PreferredAllocationResponse)
            req = dp.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=[x["uuid"] for x in inv], allocation_size=1)
            got = pref(req, timeout=5).container_responses[0].deviceIDs
            assert list(got) == O.annotations(whole)[C.ANNOT_DEVICES].split(",")
            ch.close()
            # fractional: kubelet hands arbitrary 64 CU tokens; the env is the pod's assignment
            ch, alloc = _stub(d, C.RESOURCE_GPU_CU, "Allocate", dp.AllocateRequest, dp.AllocateResponse)
            areq = dp.AllocateRequest()
            areq.container_requests.add(devices_ids=[f"{inv[1]['uuid']}::cu{k}" for k in range(64)])
            resp = alloc(areq, timeout=5).container_responses[0]
            assert resp.envs[C.ENV_ROCR_VISIBLE] == O.annotations(frac)[C.ANNOT_DEVICES]
            assert resp.envs[C.ENV_CU_MASK] == O.annotations(frac)[C.ANNOT_CU_MASK] != ""
            assert resp.envs[C.ENV_HBM_LIMIT] == "16"
            assert resp.devices[0].host_path.endswith("/kfd")
            ch.close()
            marked = O.annotations(fc.get("pods", "frac", "default"))[dp.ANNOT_ALLOCATED]
            assert marked == "gpu-cu"
            # kubelet restart: new socket -> the manager registers again
            kubelet.srv.stop(0).wait()
            os.unlink(kubelet.sock) if os.path.exists(kubelet.sock) else None
            kubelet2 = FakeKubelet(d)
            assert mgr.check_kubelet() and len(kubelet2.requests) == 3
            kubelet2.srv.stop(0)
        finally:
            mgr.stop()
            kubelet.srv.stop(0)


def test_registration_waits_for_the_kubelet():
    with tempfile.TemporaryDirectory() as d:
        fc = FakeCluster()
        fc.create("nodes", O.make_node("n1", gpus=1))
        inv = _inventory(fc.get("nodes", "n1"))
        mgr = dp.DevicePluginManager("n1", lambda: inv, client=fc, plugin_dir=d).start()   # no kubelet yet
        try:
            assert mgr.registrations == 0 and not mgr.check_kubelet()
            kubelet = FakeKubelet(d)
            assert mgr.check_kubelet() and len(kubelet.requests) == 3
            assert not mgr.check_kubelet()                  # same kubelet: no re-registration
            kubelet.srv.stop(0)
        finally:
            mgr.stop()
