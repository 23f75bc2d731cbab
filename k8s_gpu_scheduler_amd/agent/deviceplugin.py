"""Kubelet device plugin for MI355X resources (`amd.com/gpu`, `amd.com/gpu-cu`,
`amd.com/gpu-memory`).

The reference never asks the kubelet for GPUs: its pods carry no resource request and the
NVIDIA container runtime exposes every device, with CUDA_VISIBLE_DEVICES injected through
ConfigMaps (reference gpu_plugins.go:893-918, deploy/busybox/busybox.yaml).  On a real
cluster the MI355X design requests GPU shares as extended resources, so the node must
advertise them and the kubelet must hand each container its devices -- that is the
device-plugin API (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1), implemented here with
runtime-built protobuf descriptors (no protoc in the image; wire-compatible field
numbers):

* `amd.com/gpu`        one device per healthy GPU / compute partition (ID = UUID, NUMA topology);
* `amd.com/gpu-cu`     one token per compute unit (`<uuid>::cu<k>`, 256 per MI355X);
* `amd.com/gpu-memory` one token per GiB of HBM (`<uuid>::gib<k>`, 288 per MI355X).

The scheduler (GPU plugin) has already chosen the exact devices and CU slice and recorded
them on the pod (assignment annotations, written with the Binding).  The kubelet picks
token IDs on its own, so Allocate resolves WHICH pod it is allocating for the way
scheduler-driven GPU-sharing plugins do: the oldest pod bound to this node, not yet
allocated, whose request for this resource equals the number of IDs -- and returns that
pod's assignment (ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES, HSA_CU_MASK for Guaranteed
pods, the HBM cap) plus the device nodes (/dev/kfd and the GPU's /dev/dri/renderD*).
For whole GPUs GetPreferredAllocation steers the kubelet to the scheduler's choice.
Unhealthy devices (agent/health.py) are reported `Unhealthy` on ListAndWatch, so the
kubelet stops counting them as allocatable.
"""
from __future__ import annotations

import glob
import logging
import os
import threading
from concurrent import futures
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from ..api import constants as C
from ..api import objects as O
from ..utils.protodesc import field, map_entry

log = logging.getLogger(__name__)
Obj = Dict[str, Any]

API_VERSION = "v1beta1"
KUBELET_SOCKET = "/var/lib/kubelet/device-plugins/kubelet.sock"
RESOURCES = (C.RESOURCE_GPU, C.RESOURCE_GPU_CU, C.RESOURCE_GPU_MEM)
ANNOT_ALLOCATED = C.ANNOT_PREFIX + "allocated"
_F = descriptor_pb2.FieldDescriptorProto
_field = field


def _map_entry(msg: Any, name: str, num: int) -> None:
    map_entry(msg, name, num, API_VERSION)


def _build_pool() -> descriptor_pool.DescriptorPool:
    fd = descriptor_pb2.FileDescriptorProto(name="deviceplugin_v1beta1.proto", package="v1beta1", syntax="proto3")
    S, B, I64, I32, M, R = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_INT32, _F.TYPE_MESSAGE, _F.LABEL_REPEATED
    opts = fd.message_type.add(name="DevicePluginOptions")
    _field(opts, "pre_start_required", 1, B)
    _field(opts, "get_preferred_allocation_available", 2, B)
    reg = fd.message_type.add(name="RegisterRequest")
    _field(reg, "version", 1, S)
    _field(reg, "endpoint", 2, S)
    _field(reg, "resource_name", 3, S)
    _field(reg, "options", 4, M, type_name=".v1beta1.DevicePluginOptions")
    fd.message_type.add(name="Empty")
    numa = fd.message_type.add(name="NUMANode")
    _field(numa, "ID", 1, I64)
    topo = fd.message_type.add(name="TopologyInfo")
    _field(topo, "nodes", 1, M, R, ".v1beta1.NUMANode")
    dev = fd.message_type.add(name="Device")
    _field(dev, "ID", 1, S)
    _field(dev, "health", 2, S)
    _field(dev, "topology", 3, M, type_name=".v1beta1.TopologyInfo")
    lw = fd.message_type.add(name="ListAndWatchResponse")
    _field(lw, "devices", 1, M, R, ".v1beta1.Device")
    psr = fd.message_type.add(name="PreStartContainerRequest")
    _field(psr, "devices_ids", 1, S, R)
    fd.message_type.add(name="PreStartContainerResponse")
    cpr = fd.message_type.add(name="ContainerPreferredAllocationRequest")
    _field(cpr, "available_deviceIDs", 1, S, R)
    _field(cpr, "must_include_deviceIDs", 2, S, R)
    _field(cpr, "allocation_size", 3, I32)
    par = fd.message_type.add(name="PreferredAllocationRequest")
    _field(par, "container_requests", 1, M, R, ".v1beta1.ContainerPreferredAllocationRequest")
    cpa = fd.message_type.add(name="ContainerPreferredAllocationResponse")
    _field(cpa, "deviceIDs", 1, S, R)
    pal = fd.message_type.add(name="PreferredAllocationResponse")
    _field(pal, "container_responses", 1, M, R, ".v1beta1.ContainerPreferredAllocationResponse")
    car = fd.message_type.add(name="ContainerAllocateRequest")
    _field(car, "devices_ids", 1, S, R)
    ar = fd.message_type.add(name="AllocateRequest")
    _field(ar, "container_requests", 1, M, R, ".v1beta1.ContainerAllocateRequest")
    mnt = fd.message_type.add(name="Mount")
    _field(mnt, "container_path", 1, S)
    _field(mnt, "host_path", 2, S)
    _field(mnt, "read_only", 3, B)
    ds = fd.message_type.add(name="DeviceSpec")
    _field(ds, "container_path", 1, S)
    _field(ds, "host_path", 2, S)
    _field(ds, "permissions", 3, S)
    cdi = fd.message_type.add(name="CDIDevice")
    _field(cdi, "name", 1, S)
    cre = fd.message_type.add(name="ContainerAllocateResponse")
    _map_entry(cre, "envs", 1)
    _field(cre, "mounts", 2, M, R, ".v1beta1.Mount")
    _field(cre, "devices", 3, M, R, ".v1beta1.DeviceSpec")
    _map_entry(cre, "annotations", 4)
    _field(cre, "cdi_devices", 5, M, R, ".v1beta1.CDIDevice")
    are = fd.message_type.add(name="AllocateResponse")
    _field(are, "container_responses", 1, M, R, ".v1beta1.ContainerAllocateResponse")
    rs = fd.service.add(name="Registration")
    rs.method.add(name="Register", input_type=".v1beta1.RegisterRequest", output_type=".v1beta1.Empty")
    dps = fd.service.add(name="DevicePlugin")
    dps.method.add(name="GetDevicePluginOptions", input_type=".v1beta1.Empty",
                   output_type=".v1beta1.DevicePluginOptions")
    dps.method.add(name="ListAndWatch", input_type=".v1beta1.Empty", output_type=".v1beta1.ListAndWatchResponse",
                   server_streaming=True)
    dps.method.add(name="GetPreferredAllocation", input_type=".v1beta1.PreferredAllocationRequest",
                   output_type=".v1beta1.PreferredAllocationResponse")
    dps.method.add(name="Allocate", input_type=".v1beta1.AllocateRequest", output_type=".v1beta1.AllocateResponse")
    dps.method.add(name="PreStartContainer", input_type=".v1beta1.PreStartContainerRequest",
                   output_type=".v1beta1.PreStartContainerResponse")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return pool


POOL = _build_pool()


def msg(name: str) -> Any:
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(f"v1beta1.{name}"))


Empty = msg("Empty")
RegisterRequest = msg("RegisterRequest")
DevicePluginOptions = msg("DevicePluginOptions")
Device = msg("Device")
ListAndWatchResponse = msg("ListAndWatchResponse")
PreferredAllocationRequest = msg("PreferredAllocationRequest")
PreferredAllocationResponse = msg("PreferredAllocationResponse")
AllocateRequest = msg("AllocateRequest")
AllocateResponse = msg("AllocateResponse")
PreStartContainerRequest = msg("PreStartContainerRequest")
PreStartContainerResponse = msg("PreStartContainerResponse")

PLUGIN_SERVICE = "v1beta1.DevicePlugin"
REG_SERVICE = "v1beta1.Registration"


def socket_name(resource: str) -> str:
    return "amd-gpusched-" + resource.split("/", 1)[1] + ".sock"


def render_nodes(bdf: str, sysfs: str = "/sys/bus/pci/devices", dev: str = "/dev/dri") -> List[str]:
    """/dev/dri/renderD* of the GPU at PCI address `bdf` (all render nodes if unknown)."""
    if bdf:
        found = sorted(os.path.join(dev, os.path.basename(p)) for p in glob.glob(os.path.join(sysfs, bdf, "drm",
                                                                                             "renderD*")))
        if found:
            return found
    return sorted(glob.glob(os.path.join(dev, "renderD*")))


class DevicePlugin:
    """One resource's DevicePlugin service.  `inventory()` returns the agent's device
    descriptors (uuid, numa, cus, hbm_gib, healthy, bdf); `client` is the API client used to
    find the pod an Allocate is for."""

    def __init__(self, resource: str, node: str, inventory: Callable[[], List[Dict[str, Any]]], client: Any = None,
                 dev_root: str = "/dev"):
        if resource not in RESOURCES:
            raise ValueError(f"unknown resource {resource}")
        self.resource, self.node, self.inventory, self.client = resource, node, inventory, client
        self.dev_root = dev_root
        self._cv = threading.Condition()
        self._version = 0
        self._stopped = False
        self.allocations: List[Tuple[str, Dict[str, str]]] = []

    # ---------------------------------------------------------------- device list
    def device_list(self) -> List[Any]:
        out = []
        for d in self.inventory():
            health = "Healthy" if d.get("healthy", True) else "Unhealthy"
            topo = msg("TopologyInfo")(nodes=[msg("NUMANode")(ID=int(d.get("numa", 0)))])
            if self.resource == C.RESOURCE_GPU:
                ids = [d["uuid"]]
            elif self.resource == C.RESOURCE_GPU_CU:
                ids = [f"{d['uuid']}::cu{k}" for k in range(int(d.get("cus", C.MI355X_CUS)))]
            else:
                ids = [f"{d['uuid']}::gib{k}" for k in range(int(d.get("hbm_gib", C.MI355X_HBM_GIB)))]
            out.extend(Device(ID=i, health=health, topology=topo) for i in ids)
        return out

    def changed(self) -> None:
        """Inventory or health changed: every ListAndWatch stream re-sends the list."""
        with self._cv:
            self._version += 1
            self._cv.notify_all()

    def stop(self) -> None:
        with self._cv:
            self._stopped = True
            self._cv.notify_all()

    # ---------------------------------------------------------------- RPCs
    def GetDevicePluginOptions(self, request: Any, context: Any) -> Any:
        return DevicePluginOptions(pre_start_required=False,
                                   get_preferred_allocation_available=self.resource == C.RESOURCE_GPU)

    def ListAndWatch(self, request: Any, context: Any) -> Iterator[Any]:
        seen = -1
        while True:
            with self._cv:
                while self._version == seen and not self._stopped:
                    self._cv.wait(1.0)
                    if context is not None and not context.is_active():
                        return
                if self._stopped:
                    return
                seen = self._version
            yield ListAndWatchResponse(devices=self.device_list())

    def GetPreferredAllocation(self, request: Any, context: Any) -> Any:
        resp = PreferredAllocationResponse()
        for cr in request.container_requests:
            avail = list(cr.available_deviceIDs)
            want = list(cr.must_include_deviceIDs)
            pod = self._pending_pod(int(cr.allocation_size), peek=True)
            if pod is not None:
                for u in self._assigned(pod):
                    if u in avail and u not in want:
                        want.append(u)
            for u in avail:                      # fill up (kubelet requires exactly size)
                if len(want) >= cr.allocation_size:
                    break
                if u not in want:
                    want.append(u)
            resp.container_responses.add(deviceIDs=want[: cr.allocation_size])
        return resp

    def Allocate(self, request: Any, context: Any) -> Any:
        resp = AllocateResponse()
        for cr in request.container_requests:
            ids = list(cr.devices_ids)
            pod = self._pending_pod(len(ids))
            envs, devs = self._container_allocation(pod, ids)
            c = resp.container_responses.add()
            for k, v in envs.items():
                c.envs[k] = v
            for path in devs:
                c.devices.add(container_path=path, host_path=path, permissions="rw")
            if pod is not None:
                c.annotations[C.ANNOT_DEVICES] = O.annotations(pod).get(C.ANNOT_DEVICES, "")
            self.allocations.append((O.key(pod) if pod is not None else "", envs))
        return resp

    def PreStartContainer(self, request: Any, context: Any) -> Any:
        return PreStartContainerResponse()

    # ---------------------------------------------------------------- helpers
    def _request_of(self, pod: Obj) -> float:
        return float(O.pod_requests(pod).get(self.resource, 0.0))

    @staticmethod
    def _assigned(pod: Obj) -> List[str]:
        return [u for u in O.annotations(pod).get(C.ANNOT_DEVICES, "").split(",") if u]

    def _pending_pod(self, n_ids: int, peek: bool = False) -> Optional[Obj]:
        """Oldest pod bound to this node, with a scheduler assignment, not yet allocated for
        this resource, requesting exactly n_ids of it."""
        if self.client is None:
            return None
        try:
            pods, _ = self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
        except Exception as e:
            log.warning("device plugin %s: listing pods failed: %s", self.resource, e)
            return None
        done_mark = self.resource.split("/", 1)[1]
        cands = []
        for p in pods:
            ann = O.annotations(p)
            if O.is_terminal(p) or not ann.get(C.ANNOT_DEVICES):
                continue
            if done_mark in ann.get(ANNOT_ALLOCATED, "").split(","):
                continue
            if abs(self._request_of(p) - n_ids) > 1e-6:
                continue
            cands.append(p)
        if not cands:
            return None
        cands.sort(key=lambda p: (p.get("metadata", {}).get("creationTimestamp", ""), O.key(p)))
        pod = cands[0]
        if not peek:
            marks = [m for m in O.annotations(pod).get(ANNOT_ALLOCATED, "").split(",") if m] + [done_mark]
            try:
                self.client.patch("pods", O.name(pod), {"metadata": {"annotations": {
                    ANNOT_ALLOCATED: ",".join(sorted(set(marks)))}}}, "merge", namespace=O.namespace(pod))
            except Exception as e:
                log.warning("device plugin: marking %s allocated failed: %s", O.key(pod), e)
        return pod

    def _container_allocation(self, pod: Optional[Obj], ids: List[str]) -> Tuple[Dict[str, str], List[str]]:
        inv = {d["uuid"]: d for d in self.inventory()}
        if pod is not None:
            uuids = self._assigned(pod)
        else:                                    # no assignment found: the IDs' own devices
            uuids = sorted({i.split("::", 1)[0] for i in ids})
        envs = {C.ENV_ROCR_VISIBLE: ",".join(uuids),
                C.ENV_HIP_VISIBLE: ",".join(str(k) for k in range(len(uuids)))}
        if pod is not None:
            mask = O.annotations(pod).get(C.ANNOT_CU_MASK, "")
            if mask:
                envs[C.ENV_CU_MASK] = mask
            hbm = O.pod_requests(pod).get(C.RESOURCE_GPU_MEM, 0.0)
            if hbm:
                envs[C.ENV_HBM_LIMIT] = f"{hbm:g}"
        devs = [os.path.join(self.dev_root, "kfd")]
        for u in uuids:
            bdf = str(inv.get(u, {}).get("bdf", ""))
            for rn in render_nodes(bdf, dev=os.path.join(self.dev_root, "dri")):
                if rn not in devs:
                    devs.append(rn)
        return envs, devs


def _handler(plugin: DevicePlugin) -> grpc.GenericRpcHandler:
    def uu(fn, req, rep):
        return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req.FromString,
                                                   response_serializer=rep.SerializeToString)
    return grpc.method_handlers_generic_handler(PLUGIN_SERVICE, {
        "GetDevicePluginOptions": uu(plugin.GetDevicePluginOptions, Empty, DevicePluginOptions),
        "ListAndWatch": grpc.unary_stream_rpc_method_handler(
            plugin.ListAndWatch, request_deserializer=Empty.FromString,
            response_serializer=ListAndWatchResponse.SerializeToString),
        "GetPreferredAllocation": uu(plugin.GetPreferredAllocation, PreferredAllocationRequest,
                                     PreferredAllocationResponse),
        "Allocate": uu(plugin.Allocate, AllocateRequest, AllocateResponse),
        "PreStartContainer": uu(plugin.PreStartContainer, PreStartContainerRequest, PreStartContainerResponse),
    })


class DevicePluginManager:
    """Serves the three resources on Unix sockets in the kubelet's device-plugin directory
    and registers them; re-registers when the kubelet restarts (its socket is recreated)."""

    def __init__(self, node: str, inventory: Callable[[], List[Dict[str, Any]]], client: Any = None,
                 plugin_dir: str = os.path.dirname(KUBELET_SOCKET), resources=RESOURCES, dev_root: str = "/dev"):
        self.node, self.plugin_dir = node, plugin_dir
        self.plugins = {r: DevicePlugin(r, node, inventory, client, dev_root) for r in resources}
        self._servers: Dict[str, grpc.Server] = {}
        self._kubelet_id: Optional[Tuple[int, int]] = None
        self.registrations = 0

    @property
    def kubelet_socket(self) -> str:
        return os.path.join(self.plugin_dir, os.path.basename(KUBELET_SOCKET))

    def start(self) -> "DevicePluginManager":
        for r, p in self.plugins.items():
            path = os.path.join(self.plugin_dir, socket_name(r))
            if os.path.exists(path):
                os.unlink(path)
            srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
            srv.add_generic_rpc_handlers((_handler(p),))
            srv.add_insecure_port(f"unix://{path}")
            srv.start()
            self._servers[r] = srv
        try:
            self.register()
        except Exception as e:        # kubelet not up yet: run_forever keeps retrying
            log.warning("device plugin registration deferred: %s", e)
        return self

    def register(self, timeout_s: float = 5.0) -> None:
        with grpc.insecure_channel(f"unix://{self.kubelet_socket}") as ch:
            call = ch.unary_unary(f"/{REG_SERVICE}/Register", request_serializer=RegisterRequest.SerializeToString,
                                  response_deserializer=Empty.FromString)
            for r, p in self.plugins.items():
                opts = p.GetDevicePluginOptions(None, None)
                call(RegisterRequest(version=API_VERSION, endpoint=socket_name(r), resource_name=r, options=opts),
                     timeout=timeout_s)
                self.registrations += 1
        st = os.stat(self.kubelet_socket)
        self._kubelet_id = (st.st_ino, st.st_ctime_ns)

    def check_kubelet(self) -> bool:
        """Re-register after a kubelet restart (new socket inode); returns True if it did."""
        try:
            st = os.stat(self.kubelet_socket)
        except FileNotFoundError:
            return False
        if self._kubelet_id == (st.st_ino, st.st_ctime_ns):
            return False
        self.register()
        return True

    def changed(self) -> None:
        for p in self.plugins.values():
            p.changed()

    def stop(self) -> None:
        for p in self.plugins.values():
            p.stop()
        for srv in self._servers.values():
            srv.stop(grace=0.5)
        self._servers.clear()

    def run_forever(self, poll_s: float = 5.0, stop: Optional[threading.Event] = None) -> None:
        stop = stop or threading.Event()
        while not stop.wait(poll_s):
            try:
                self.check_kubelet()
            except Exception as e:
                log.warning("kubelet re-registration failed: %s", e)
        self.stop()
