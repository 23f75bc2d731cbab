"""`gpu-sched` command line: every binary of the reference as one entry point.

  gpu-sched scheduler   --config scheduler-config.yaml [--kubeconfig K] [--v 3]
                        (reference: gpu-sched --config=/config/scheduler-config.yaml --v=3,
                         deploy/scheduler.yaml:63-66; leader election from the config)
  gpu-sched extender    --config ... --port 8888   (kube-scheduler extender front-end)
  gpu-sched recommender --port 50051               (reference recom_server.py; env
                         CONFIGURATIONS_DATA_PATH / INTERFERENCE_DATA_PATH / PORT / JOB_DELAY)
  gpu-sched agent       --node $NODE_NAME          (reference profiler DaemonSet)
  gpu-sched redisctl    -l/--list -f/--flush -c/--config   (reference redisCtl.go:22-26)
  gpu-sched resize-webhook --redis host:port --port 8443 --tls-cert c --tls-key k  (config 5)
  gpu-sched devquery                               (reference gpu_profiling.cpp, all devices)
  gpu-sched profile     (measure the MI355X configuration/interference tables)
  gpu-sched bench       (pod-arrival benchmark; same as bench.py)
  gpu-sched fake-cluster --port 6443               (HTTP fake apiserver for local runs)
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import socket
import sys
import threading
import time
from typing import List, Optional

from ..api import constants as C


def _client(kubeconfig: str = "", fake_url: str = "", master: str = ""):
    """REST client: a fake apiserver URL as is; else the kubeconfig / in-cluster config, with
    `master` (kube-scheduler's --master) replacing its server address."""
    from ..kube.rest import RestClient, RestConfig
    if fake_url:
        return RestClient(RestConfig(fake_url))
    if master:
        try:
            base = RestClient.auto(kubeconfig).cfg
        except Exception:
            return RestClient(RestConfig(master))
        base.host = master
        return RestClient(base)
    return RestClient.auto(kubeconfig)


def _endpoints(args, client):
    from ..utils.discovery import Endpoints
    ep = Endpoints.from_env()
    if getattr(args, "redis", ""):
        ep.redis = args.redis
    if getattr(args, "recommender", ""):
        ep.recommender = args.recommender
    if not (ep.redis and ep.recommender) and not getattr(args, "no_discovery", False):
        try:
            ep.discover(client)
        except Exception as e:
            logging.warning("service discovery failed: %s", e)
    return ep


def _build_scheduler(args, client):
    from ..framework.config import default_gpu_config, load_config
    from ..framework.scheduler import Scheduler
    from ..plugins import full_registry
    from ..telemetry.cache import TelemetryCache
    cfg = load_config(args.config) if args.config else default_gpu_config({})
    ep = _endpoints(args, client)
    prom = getattr(args, "prometheus", "") or ep.prometheus
    for prof in cfg.profiles:
        gargs = prof.plugin_config.setdefault(C.PLUGIN_NAME, {})
        if ep.redis and not gargs.get("redis"):
            gargs["redis"] = ep.redis
            gargs.setdefault("redis_password", ep.redis_password)
        if ep.recommender and not gargs.get("recommender"):
            gargs["recommender"] = ep.recommender
        if prom and not gargs.get("prometheus"):
            gargs["prometheus"] = prom
        prom = prom or gargs.get("prometheus", "")
    # one live-telemetry cache shared by every profile's GPU plugin, filled by the poller
    tele = TelemetryCache(stale_s=getattr(args, "telemetry_stale", 10.0))
    sched = Scheduler(client, cfg, full_registry(), extras={"telemetry": tele})
    sched.telemetry_poller = _telemetry_poller(args, tele, prom)
    return cfg, sched


def _telemetry_poller(args, cache, prometheus: str):
    """Background reader of the agents' GPU series (Prometheus instant queries, or direct
    exporter scrapes with --telemetry-scrape); None when neither is configured."""
    from ..telemetry.poller import TelemetryPoller, make_source
    src = make_source(prometheus, getattr(args, "telemetry_scrape", ""))
    if src is None:
        logging.warning("no Prometheus / exporter endpoint: Score runs without live telemetry")
        return None
    return TelemetryPoller(cache, src, getattr(args, "telemetry_period", 2.0))


def cmd_scheduler(args) -> int:
    from ..kube.leader import LeaderElector
    client = _client(args.kubeconfig, args.fake_apiserver, getattr(args, "master", ""))
    cfg, sched = _build_scheduler(args, client)
    # kube-scheduler's command-line overrides of the config file
    if getattr(args, "leader_elect", None) is not None:
        cfg.leader_election.leader_elect = args.leader_elect
    if getattr(args, "leader_elect_resource_name", ""):
        cfg.leader_election.resource_name = args.leader_elect_resource_name
    if getattr(args, "leader_elect_resource_namespace", ""):
        cfg.leader_election.resource_namespace = args.leader_elect_resource_namespace
    http = None
    if args.metrics_port:
        from ..telemetry.exporter import GpuExporter, SchedulerHTTP, attach_scheduler_metrics
        exp = GpuExporter(os.getenv("NODE_NAME", socket.gethostname()), exporter_pod=os.getenv("POD_NAME", ""))
        attach_scheduler_metrics(exp, sched)
        http = SchedulerHTTP(exp, sched, args.metrics_port, getattr(args, "bind_address", "0.0.0.0")).start()
        logging.info("scheduler /metrics /healthz /livez /readyz on :%d", http.port)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    if cfg.leader_election.leader_elect:
        le = cfg.leader_election
        ident = f"{socket.gethostname()}_{os.getpid()}"
        elector = LeaderElector(client, le.resource_name, le.resource_namespace, ident, le.lease_duration_s,
                                le.renew_deadline_s, le.retry_period_s, on_started_leading=sched.start,
                                on_stopped_leading=stop.set)
        elector.start()
    else:
        sched.start()
    if sched.telemetry_poller is not None:
        sched.telemetry_poller.start()
    ctrls = _partition_controllers(sched)
    try:
        while not stop.is_set():
            if ctrls and (not cfg.leader_election.leader_elect or sched._thread is not None):
                for c in ctrls:         # only the leader (once its loop runs) re-partitions
                    c.start()
            stop.wait(1.0)
    except KeyboardInterrupt:
        pass
    for c in ctrls:
        c.stop()
    if sched.telemetry_poller is not None:
        sched.telemetry_poller.stop()
    sched.stop()
    if http is not None:
        http.stop()
    return 0


def _partition_controllers(sched):
    """The GPU plugin's partition controllers (plugins.gpu.partitioner), one per profile."""
    out = []
    for fw in sched.frameworks.values():
        try:
            p = fw.plugin(C.PLUGIN_NAME)
        except Exception:
            continue
        if p is not None and getattr(p, "partitioner", None) is not None:
            out.append(p.partitioner)
    return out


def cmd_extender(args) -> int:
    from ..framework.extender import Extender, ExtenderServer
    client = _client(args.kubeconfig, args.fake_apiserver)
    _, sched = _build_scheduler(args, client)
    sched.start_informers()
    if sched.telemetry_poller is not None:
        sched.telemetry_poller.start()
    srv = ExtenderServer(Extender(sched), "0.0.0.0", args.port).start()
    logging.info("extender listening on %s", srv.url)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()
    return 0


def cmd_recommender(args) -> int:
    from ..recommender.service import RecommenderService
    svc = RecommenderService.from_env(kind=args.model)
    if args.redis:
        from ..store import schema
        from ..store.resp import Redis
        r = Redis.connect(args.redis, args.redis_password)
        svc.history_source = lambda pod: schema.read_history(r, pod)
        svc.store = r                   # persist / restore trained model versions
    svc.train()
    svc.start_retrain_loop()
    port = int(os.getenv("PORT", args.port))
    server, bound = svc.make_server(port, args.workers)
    logging.info("recommender serving on :%d", bound)
    server.wait_for_termination()
    return 0


def cmd_resize_webhook(args) -> int:
    """Mutating admission webhook that right-sizes fractional GPU requests from the
    per-workload history in Redis (BASELINE config 5; recommender/admission.py)."""
    from ..recommender.admission import AdmissionServer, RedisHistory, ResizeAdmission
    from ..store.resp import Redis
    if not args.redis:
        logging.error("--redis is required (history store)")
        return 2
    hist = RedisHistory(Redis.connect(args.redis, args.redis_password))
    preds = None
    if args.recommender:
        from ..recommender.client import CachedPredictions, RecommenderClient
        cp = CachedPredictions(RecommenderClient(args.recommender))
        preds = cp.configurations
    adm = ResizeAdmission(hist.read, preds, min_samples=args.min_samples, shrink_only=args.shrink_only)
    routes = {}
    if args.profile:
        # per-pod rocprofv3 injection (agent.profile_webhook): /profile alone, and chained
        # after the resize on /mutate so a pod gets both with one webhook call
        from ..agent.profile_webhook import ChainAdmission, ProfileInjector
        inj = ProfileInjector(rocprof=args.rocprof, host_dir=args.profile_host_dir)
        routes["/profile"] = inj
        adm = ChainAdmission(adm, inj)
    srv = AdmissionServer(adm, "0.0.0.0", args.port, args.tls_cert, args.tls_key, routes=routes).start()
    logging.info("resize webhook on %s", srv.url)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()
    return 0


def _corun_sender(addr: str):
    """RecommenderClient.observe_corun for the agent's co-run observer (None: no recommender)."""
    if not addr:
        return None
    from ..recommender.client import RecommenderClient
    cl = RecommenderClient(addr)
    return cl.observe_corun


def _fabric_prober(args):
    """Per-pair xGMI copy-rate probe for the agent (agent.fabric): on real devices unless
    --fabric-probe off; never with --synthetic GPUs."""
    if args.fabric_probe == "off" or args.synthetic:
        return None
    from ..agent.fabric import FabricProber
    return FabricProber()


def _set_checker(args):
    """RCCL checks of the GPU sets multi-GPU pods ran on (agent.probes): with the fabric probe."""
    if args.fabric_probe == "off" or args.synthetic or args.set_checks == "off":
        return None
    from ..agent.probes import SetChecker
    return SetChecker()


def cmd_agent(args) -> int:
    from ..agent.agent import NodeAgent
    from ..agent.devices import best_source, synthetic_node
    from ..store.resp import Redis
    from ..telemetry.exporter import GpuExporter
    node = args.node or os.getenv("NODE_NAME") or socket.gethostname()
    client = None
    try:
        client = _client(args.kubeconfig, args.fake_apiserver)
    except Exception as e:
        logging.warning("no apiserver access (%s); partition reconcile disabled", e)
    ep = _endpoints(args, client) if client is not None else None
    addr = args.redis or (ep.redis if ep else "")
    if not addr:
        logging.error("Redis not found")
        return 1
    redis = Redis.connect(addr, args.redis_password)
    src = synthetic_node(args.synthetic, node=node) if args.synthetic else best_source()
    if args.synthetic and args.synthetic_samples:
        # scripted telemetry for a synthetic node: JSON list of per-device sample dicts
        # ({"index": i, "gfx_activity": 95, "vram_used_mb": ...}, amd-smi units)
        src._samples = json.loads(args.synthetic_samples)
    exp = GpuExporter(node, os.getenv("POD_NAME", "amd-gpu-exporter"), dcgm_compat=args.dcgm_compat)
    if args.metrics_port:
        exp.serve(args.metrics_port)
    # amd-smi reports HOST pids: attribute them through the host's /proc (the DaemonSet
    # mounts it at /host/proc) unless told otherwise
    from ..agent.agent import pod_of_pid
    proc_root = args.proc_root or ("/host/proc" if os.path.isdir("/host/proc") else "/proc")
    agent = NodeAgent(node, redis, src, client, args.poll, exporter=exp, evict_unhealthy=args.evict_unhealthy,
                      evict_hbm_overuse=args.evict_hbm_overuse, drain_timeout_s=args.drain_timeout,
                      hbm_tolerance_gib=args.hbm_tolerance, host_proc=proc_root, profile_dir=args.profile_dir,
                      partition_dry_run=args.partition_dry_run,
                      fabric=_fabric_prober(args), corun_send=_corun_sender(args.corun_recommender),
                      background_probes=True, set_checks=_set_checker(args),
                      pod_resolver=lambda pid: pod_of_pid(pid, proc_root))
    mgr = None
    if args.device_plugin:
        # kubelet device plugin for amd.com/gpu, amd.com/gpu-cu, amd.com/gpu-memory
        from ..agent.deviceplugin import DevicePluginManager
        agent.publish(force=True)
        mgr = DevicePluginManager(node, agent.inventory, client=client, plugin_dir=args.device_plugin_dir).start()
        agent.on_inventory_change.append(mgr.changed)
        threading.Thread(target=mgr.run_forever, name="device-plugin", daemon=True).start()
    if args.once:
        agent.step()
        if agent.probes is not None:
            agent.probes.tick()
        if mgr is not None:
            mgr.stop()
        return 0
    agent.run()
    return 0


def cmd_redisctl(args) -> int:
    """List every key/value and/or flush (reference redisCtl.go:21-80)."""
    from ..store.resp import Redis
    addr = args.redis
    if not addr:
        client = _client(args.config)
        ep = _endpoints(args, client)
        addr = ep.redis
    if not addr:
        print("Redis not found", file=sys.stderr)
        return 1
    r = Redis.connect(addr, args.redis_password)
    if args.list:
        for k in r.get_keys():
            try:
                print(f"{k}: {r.get(k)}")
            except Exception:
                print(f"{k}: <{r.backend.execute('TYPE', k) if hasattr(r.backend, 'execute') else 'non-string'}>")
    if args.flush:
        r.flush()
    return 0


def cmd_devquery(args) -> int:
    from .. import _native
    h = _native.hip(required=False)
    out = {"hip": h.query_all() if h is not None else [], "smi": None}
    s = _native.smi()
    if s is not None:
        x = s.Smi()
        if x.init():
            out["smi"] = {"devices": x.devices(), "topology": x.topology(), "samples": x.sample()}
            x.shutdown()
        else:
            out["smi"] = {"error": x.error()}
    print(json.dumps(out, indent=1, default=str))
    return 0


def cmd_profile(args) -> int:
    from ..models.profile import main as prof_main
    return prof_main(args.rest)


def cmd_bench(args) -> int:
    from ..parallel.podbench import main as bench_main
    bench_main(args.rest)
    return 0


def cmd_fake_cluster(args) -> int:
    from ..api import objects as O
    from ..kube.fake_apiserver import FakeApiServer
    srv = FakeApiServer(port=args.port).start()
    for i in range(args.nodes):
        srv.cluster.create("nodes", O.make_node(f"mi355x-node-{i}", gpus=args.gpus))
    print(srv.url, flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()
    return 0


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="gpu-sched", description="MI355X-native Kubernetes GPU scheduler")
    p.add_argument("--v", type=int, default=2, help="log verbosity (klog style)")
    sub = p.add_subparsers(dest="cmd", required=True)

    def common(sp):
        sp.add_argument("--kubeconfig", default="")
        sp.add_argument("--fake-apiserver", default="", help="URL of a fake apiserver")
        sp.add_argument("--redis", default="")
        sp.add_argument("--redis-password", default=C.REDIS_PASSWORD)
        sp.add_argument("--recommender", default="")
        sp.add_argument("--no-discovery", action="store_true")

    def telemetry(sp):
        sp.add_argument("--prometheus", default="", help="Prometheus URL for the live GPU telemetry poller")
        sp.add_argument("--telemetry-scrape", default="",
                        help="comma-separated agent exporter /metrics URLs, scraped directly (no Prometheus)")
        sp.add_argument("--telemetry-period", type=float, default=2.0, help="telemetry poll period (s)")
        sp.add_argument("--telemetry-stale", type=float, default=10.0,
                        help="samples older than this are ignored by Score (s)")

    s = sub.add_parser("scheduler")
    common(s)
    telemetry(s)
    s.add_argument("--config", default="")
    s.add_argument("--metrics-port", "--port", type=int, default=10251,
                   help="HTTP port of /metrics (pods scheduled, latency, per-extension-point means) and "
                        "/healthz /livez /readyz; 0 = off")
    s.add_argument("--bind-address", default="0.0.0.0")
    s.add_argument("--master", default="", help="apiserver URL (overrides the kubeconfig's server)")
    s.add_argument("--leader-elect", default=None, type=lambda v: str(v).lower() in ("1", "true", "yes"),
                   help="override the config's leaderElection.leaderElect (true/false)")
    s.add_argument("--leader-elect-resource-name", default="")
    s.add_argument("--leader-elect-resource-namespace", default="")
    s.set_defaults(fn=cmd_scheduler)
    s = sub.add_parser("extender")
    common(s)
    telemetry(s)
    s.add_argument("--config", default="")
    s.add_argument("--port", type=int, default=8888)
    s.set_defaults(fn=cmd_extender)
    s = sub.add_parser("recommender")
    s.add_argument("--port", type=int, default=C.RECOMMENDER_PORT)
    s.add_argument("--workers", type=int, default=C.RECOMMENDER_WORKERS)
    s.add_argument("--model", default="iterative", choices=["iterative", "svd", "als"])
    s.add_argument("--redis", default="")
    s.add_argument("--redis-password", default=C.REDIS_PASSWORD)
    s.set_defaults(fn=cmd_recommender)
    s = sub.add_parser("resize-webhook")
    s.add_argument("--redis", default="")
    s.add_argument("--redis-password", default=C.REDIS_PASSWORD)
    s.add_argument("--recommender", default="")
    s.add_argument("--port", type=int, default=8443)
    s.add_argument("--tls-cert", default="")
    s.add_argument("--tls-key", default="")
    s.add_argument("--min-samples", type=int, default=3)
    s.add_argument("--shrink-only", action="store_true")
    s.add_argument("--profile", action="store_true",
                   help="also wrap opted-in pods (label gpu-scheduler.amd.com/profile=trace|pmc) in rocprofv3")
    s.add_argument("--rocprof", default="rocprofv3", help="rocprofv3 path inside the pods' images")
    s.add_argument("--profile-host-dir", default="/var/lib/gpusched/prof")
    s.set_defaults(fn=cmd_resize_webhook)
    s = sub.add_parser("agent")
    common(s)
    s.add_argument("--node", default="")
    s.add_argument("--poll", type=float, default=C.PROFILER_POLL_S)
    s.add_argument("--metrics-port", type=int, default=9400)
    s.add_argument("--dcgm-compat", action="store_true")
    s.add_argument("--synthetic", type=int, default=0, help="fake N GPUs (no hardware)")
    s.add_argument("--synthetic-samples", default="", help="scripted telemetry of the synthetic GPUs (JSON list)")
    s.add_argument("--once", action="store_true")
    s.add_argument("--device-plugin", action="store_true",
                   help="also serve the kubelet device plugin (amd.com/gpu, gpu-cu, gpu-memory)")
    s.add_argument("--device-plugin-dir", default="/var/lib/kubelet/device-plugins")
    s.add_argument("--evict-unhealthy", action="store_true",
                   help="delete pods assigned to a GPU that turns unhealthy (controllers reschedule them)")
    s.add_argument("--evict-hbm-overuse", action="store_true",
                   help="evict (Eviction API, PodDisruptionBudgets apply) pods whose processes hold more VRAM "
                        "than their amd.com/gpu-memory share")
    s.add_argument("--set-checks", default="auto", choices=["auto", "off"],
                   help="RCCL all-reduce check of each multi-GPU pod's GPU set once it is idle again "
                        "(agent.probes); a set below par is published in the topology's bad_sets")
    s.add_argument("--fabric-probe", default="auto", choices=["auto", "off"],
                   help="measure every GPU pair's copy rate (child process, idle GPUs only) at start-up and "
                        "after partition changes; published with the topology for multi-GPU placement")
    s.add_argument("--partition-dry-run", action="store_true",
                   help="check partition requests (capabilities, idleness) but only record the amd-smi calls "
                        "that would apply them (node annotation partition-state: dry-run)")
    s.add_argument("--profile-dir", default="",
                   help="hostPath where profiled pods' rocprofv3 output lands (mounted from /var/lib/gpusched/prof; "
                        "see the resize webhook's --profile): finished runs go to the workload history in Redis")
    s.add_argument("--corun-recommender", default=os.getenv("RECOMMENDER_ADDR", ""),
                   help="recommender host:port: with --profile-dir, profiled pods that overlapped on one GPU are sent "
                        "as co-run observations (ObserveCorun) for its online co-run model")
    s.add_argument("--hbm-tolerance", type=float, default=0.5,
                   help="GiB over a pod's HBM share before it counts as overuse; must cover the HIP runtime's "
                        "per-process VRAM (~0.3 GiB on MI355X), which amd-smi counts and the request does not")
    s.add_argument("--proc-root", default="", help="host /proc for pid -> pod attribution (default /host/proc)")
    s.add_argument("--drain-timeout", type=float, default=300.0,
                   help="seconds a partition request waits for the GPUs to go idle before it is refused")
    s.set_defaults(fn=cmd_agent)
    s = sub.add_parser("redisctl")
    s.add_argument("-l", "--list", action="store_true", help="List redis' data")
    s.add_argument("-f", "--flush", action="store_true", help="Flush redis database")
    s.add_argument("-c", "--config", default=os.path.expanduser("~/.kube/config"), help="Kubernetes config path")
    s.add_argument("--redis", default="")
    s.add_argument("--redis-password", default=C.REDIS_PASSWORD)
    s.add_argument("--no-discovery", action="store_true")
    s.set_defaults(fn=cmd_redisctl)
    s = sub.add_parser("devquery")
    s.set_defaults(fn=cmd_devquery)
    s = sub.add_parser("profile")
    s.add_argument("rest", nargs=argparse.REMAINDER)
    s.set_defaults(fn=cmd_profile)
    s = sub.add_parser("bench")
    s.add_argument("rest", nargs=argparse.REMAINDER)
    s.set_defaults(fn=cmd_bench)
    s = sub.add_parser("fake-cluster")
    s.add_argument("--port", type=int, default=6443)
    s.add_argument("--nodes", type=int, default=1)
    s.add_argument("--gpus", type=int, default=8)
    s.set_defaults(fn=cmd_fake_cluster)
    return p


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if args.v >= 4 else logging.INFO if args.v >= 2 else logging.WARNING,
                        format="%(asctime)s %(levelname).1s %(name)s] %(message)s")
    return int(args.fn(args) or 0)


if __name__ == "__main__":
    sys.exit(main())
