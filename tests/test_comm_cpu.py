"""Host-side pieces of the communicator (no GPU needed): the TCP bootstrap
hands every rank rank 0's RCCL unique id, and the TCP transport's star
connects (swps_comm_create_tcp: a host-only object until an exchange runs).
Ranks are fresh processes (spawn)."""
import ctypes
import multiprocessing as mp
import socket

import pytest


def _port():
    from conftest import free_port
    return free_port()


def _boot(rank, world, port, q):
    from swiftmpi_amd import capi
    uid = (ctypes.c_uint8 * capi.COMM_ID_BYTES)()
    rc = capi.lib().swps_comm_bootstrap_tcp(b"127.0.0.1", port, rank, world, 20000, uid)
    q.put((rank, rc, bytes(uid), capi.lib().swps_last_error().decode()))


def _tcp(rank, world, port, q):
    from swiftmpi_amd import capi
    h = ctypes.c_void_p()
    rc = capi.lib().swps_comm_create_tcp(b"127.0.0.1", port, rank, world, 0, 20000, ctypes.byref(h))
    r, w = ctypes.c_int32(), ctypes.c_int32()
    if rc == 0:
        capi.lib().swps_comm_info(h, ctypes.byref(r), ctypes.byref(w))
        capi.lib().swps_comm_destroy(h)
    q.put((rank, rc, r.value, w.value, capi.lib().swps_last_error().decode()))


def _run(target, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    return out


def test_bootstrap_tcp_shares_rank0_id(lib):
    out = _run(_boot, 3)
    if out[0][1] != 0:
        pytest.skip("ncclGetUniqueId unavailable here: %s" % out[0][3])
    assert all(o[1] == 0 for o in out), out
    assert len({o[2] for o in out}) == 1 and any(out[0][2])


def test_tcp_transport_star_connects(lib):
    out = _run(_tcp, 3)
    assert all(o[1] == 0 for o in out), out
    assert [(o[2], o[3]) for o in out] == [(0, 3), (1, 3), (2, 3)]


def test_comm_argument_errors(lib):
    from swiftmpi_amd import capi
    h = ctypes.c_void_p()
    assert capi.lib().swps_comm_create_tcp(b"127.0.0.1", 0, 0, 2, 0, 100, ctypes.byref(h)) == -5  # port 0
    assert capi.lib().swps_comm_create_tcp(b"not-an-ip", 29999, 1, 2, 0, 100, ctypes.byref(h)) == -5
    uid = (ctypes.c_uint8 * capi.COMM_ID_BYTES)()
    assert capi.lib().swps_comm_bootstrap_tcp(b"127.0.0.1", 29999, 2, 2, 100, uid) == -5
