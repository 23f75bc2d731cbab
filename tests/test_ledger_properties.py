"""Property / concurrency tests of the device ledger (a hypothesis-based
concurrency test of Reserve/Unreserve).  Invariants after any interleaving of reserve /
release from several threads: no CU-slice unit is held by two pods, HBM accounting equals
the sum of the holders, find_units only returns free aligned runs, and the pod index
agrees with the per-device state."""
import threading

from hypothesis import given, settings
from hypothesis import strategies as st

from k8s_gpu_scheduler_amd.plugins.gpu.devices import Device, DeviceLedger

NODE = "n"


def _ledger(gpus=2):
    led = DeviceLedger()
    led.set_devices(NODE, [Device(f"GPU-{g}", NODE, g) for g in range(gpus)])
    return led


def _check(led: DeviceLedger) -> None:
    for stt in led.devices(NODE):
        owner = [None] * stt.device.units
        hbm = 0.0
        for key, use in stt.pods.items():
            u0, n = use.units
            for u in range(u0, u0 + n):
                assert owner[u] is None, f"unit {u} of {stt.device.uuid} double-booked"
                owner[u] = key
            hbm += use.hbm_gib
            assert led.placement(key) is not None
        assert [o is not None for o in owner] == stt.used_units
        assert abs(hbm - stt.hbm_used) < 1e-6
        for n in (1, 2, 4, 8):
            u0 = stt.find_units(n)
            if u0 is not None:
                assert u0 % n == 0 and not any(stt.used_units[u0:u0 + n])


ops = st.lists(st.tuples(st.sampled_from(["reserve", "release"]), st.integers(0, 15),
                         st.sampled_from([1, 2, 4, 8]), st.integers(0, 1), st.floats(0, 100)), max_size=60)


@settings(max_examples=150, deadline=None)
@given(ops)
def test_ledger_sequential_invariants(seq):
    led = _ledger()
    for op, pid, n, gpu, hbm in seq:
        key = f"default/p{pid}"
        if op == "reserve":
            stt = led.devices(NODE)[gpu]
            u0 = stt.find_units(n)
            if u0 is not None:
                led.reserve(NODE, key, f"p{pid}", 0.0, [(stt.device.uuid, u0, n, hbm, False)])
        else:
            led.release(key)
        _check(led)


@settings(max_examples=30, deadline=None)
@given(st.lists(ops, min_size=2, max_size=4))
def test_ledger_concurrent_invariants(per_thread):
    """Threads race find_units -> reserve (the scheduler's assume) and release; reserve is
    all-or-nothing under the ledger lock, so a lost race fails cleanly instead of
    double-booking."""
    led = _ledger()
    barrier = threading.Barrier(len(per_thread))

    def worker(t, seq):
        barrier.wait()
        for op, pid, n, gpu, hbm in seq:
            key = f"default/t{t}p{pid}"
            if op == "reserve":
                stt = led.devices(NODE)[gpu]
                u0 = stt.find_units(n)
                if u0 is not None:
                    led.reserve(NODE, key, key, 0.0, [(stt.device.uuid, u0, n, hbm, False)])
            else:
                led.release(key)
    ths = [threading.Thread(target=worker, args=(t, s)) for t, s in enumerate(per_thread)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    _check(led)
