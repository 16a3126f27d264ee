"""Communicators for the library's own key-sharded table (swps_comm_*,
swps_table_route): RCCL from a bootstrap, or a host transport whose
all-gather / all-to-all-v callbacks run over a torch.distributed process
group (gloo: several ranks sharing one GPU in tests — RCCL refuses that).

The library issues the exchanges itself (include/swps.h "communicator");
this module only builds the handle."""
import ctypes
import os
import traceback

import numpy as np

from . import capi
from .capi import check

IPC_CHANNELS = 8     # swps_comm.hip kIpcCh: workgroups per peer and direction
IPC_MIN_PART = 4096  # swps_comm.hip kIpcMinPart: a segment's least per-channel part


class Comm:
    def __init__(self, handle, rank, world, keep=()):
        self.h = handle
        self.rank, self.world = rank, world
        self._keep = keep  # ctypes callbacks must outlive the handle

    @classmethod
    def rccl(cls, rank, world, device=0, addr="127.0.0.1", port=29611, timeout_ms=60000):
        """RCCL communicator; rank 0 serves the unique id over TCP (addr:port)."""
        uid = (ctypes.c_uint8 * capi.COMM_ID_BYTES)()
        check(capi.lib().swps_comm_bootstrap_tcp(addr.encode(), port, rank, world, timeout_ms, uid))
        h = ctypes.c_void_p()
        check(capi.lib().swps_comm_create_rccl(uid, rank, world, device, ctypes.byref(h)))
        return cls(h, rank, world)

    @classmethod
    def tcp(cls, rank, world, device=0, addr="127.0.0.1", port=29612, timeout_ms=60000):
        """The library's own TCP star transport (several ranks may share a GPU)."""
        h = ctypes.c_void_p()
        check(capi.lib().swps_comm_create_tcp(addr.encode(), port, rank, world, device, timeout_ms, ctypes.byref(h)))
        return cls(h, rank, world)

    @classmethod
    def host(cls, group=None, device=0):
        """Host transport over a torch.distributed group (gloo)."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)

        def allgather(_ctx, src, dst, nbytes):
            try:
                t = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(src)).copy())
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(outs, t, group=group)
                flat = torch.cat(outs).numpy()
                ctypes.memmove(dst, flat.ctypes.data, flat.size)
                return 0
            except Exception:  # noqa: BLE001 — an exception must not cross the C boundary
                traceback.print_exc()
                return 1

        def alltoallv(_ctx, src, sbytes, dst, rbytes):
            try:
                sb = [int(sbytes[r]) for r in range(world)]
                rb = [int(rbytes[r]) for r in range(world)]
                n = sum(sb)
                send = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(src))[:n].copy())
                recv = torch.empty(sum(rb), dtype=torch.uint8)
                dist.all_to_all_single(recv, send, rb, sb, group=group)
                if recv.numel():
                    ctypes.memmove(dst, recv.numpy().ctypes.data, recv.numel())
                return 0
            except Exception:  # noqa: BLE001
                traceback.print_exc()
                return 1

        ag = capi.ALLGATHER_FN(allgather)
        a2a = capi.ALLTOALLV_FN(alltoallv)
        tr = capi.Transport(None, ag, a2a)
        h = ctypes.c_void_p()
        check(capi.lib().swps_comm_create_host(ctypes.byref(tr), rank, world, device, ctypes.byref(h)))
        return cls(h, rank, world, keep=(ag, a2a, tr))

    def transport(self):
        """("rccl" | "tcp" | "host", the rank count the transport reports — RCCL: ncclCommCount)."""
        k, n = ctypes.c_int32(), ctypes.c_int32()
        check(capi.lib().swps_comm_transport(self.h, ctypes.byref(k), ctypes.byref(n)))
        return {1: "rccl", 2: "tcp", 3: "host"}[k.value], n.value

    def enable_ipc(self, slot_bytes=0):
        """Collective: later exchanges move device to device through IPC-mapped peer inboxes
        (swps_comm_enable_ipc; the ranks of one node)."""
        check(capi.lib().swps_comm_enable_ipc(self.h, int(slot_bytes)))
        return self

    def ipc_info(self):
        """{"enabled", "slot_bytes", "exchanges", "bytes_remote"} of the IPC exchange."""
        out = (ctypes.c_uint64 * 4)()
        check(capi.lib().swps_comm_ipc_info(self.h, out))
        return dict(zip(("enabled", "slot_bytes", "exchanges", "bytes_remote"), (int(v) for v in out)))

    def alltoallv(self, send, send_counts, recv, recv_counts, stream=None):
        """Collective all-to-all-v of two device tensors (counts in elements, per rank) on
        `stream` (torch's current stream by default)."""
        import torch
        es = send.element_size()
        sb = (ctypes.c_uint64 * self.world)(*(int(n) * es for n in send_counts))
        rb = (ctypes.c_uint64 * self.world)(*(int(n) * es for n in recv_counts))
        s = (stream or torch.cuda.current_stream()).cuda_stream
        check(capi.lib().swps_comm_alltoallv(self.h, ctypes.c_void_p(send.data_ptr()), sb,
                                             ctypes.c_void_p(recv.data_ptr()), rb, ctypes.c_void_p(s)))

    def canary(self):
        """One IPC exchange with every segment size class (17 B .. 2.5 inbox slots: the multi-round
        path) and a per-(source, destination) byte pattern, checked on the device.  Returns
        (ok, report): report lists, per source rank whose segment arrived wrong, where — the peer,
        the channel and round of the exchange that carried the first wrong byte, its byte offset in
        that peer's segment and in the receive buffer, the 8-byte words expected and received there,
        and the count of wrong bytes — so a cross-device ordering fault can be located from one
        record.  SWPS_IPC_DIAG_CORRUPT=<rank>:<offset> flips the received byte at <offset> on rank
        <rank> before the check (a test of this report)."""
        import torch
        slot = self.ipc_info()["slot_bytes"]
        sizes = [1024, 5 * slot // 2 + 7, 4099, slot, 64 << 10, 3 * slot // 2, 17, 1 << 20]
        rank, world = self.rank, self.world

        def size(src, dst):
            return sizes[(src * 3 + dst) % len(sizes)]

        def seg(src, dst):
            n = size(src, dst)
            return (torch.arange(n, dtype=torch.int64, device="cuda") * (2 * src + 3) + 7 * dst).to(torch.uint8)
        send = torch.cat([seg(rank, d) for d in range(world)])
        want = torch.cat([seg(s_, rank) for s_ in range(world)])
        recv = torch.zeros_like(want)
        self.alltoallv(send, [size(rank, d) for d in range(world)], recv, [size(s_, rank) for s_ in range(world)])
        torch.cuda.synchronize()
        self.check()
        inj = os.environ.get("SWPS_IPC_DIAG_CORRUPT")
        if inj:
            r_, o_ = (int(x) for x in inj.split(":"))
            if r_ == rank:
                recv[o_] ^= 0xFF
        bad = recv != want
        if not bool(bad.any()):
            return True, []
        report = []
        sub = slot // IPC_CHANNELS
        base = 0
        for src in range(world):
            n = size(src, rank)
            b = bad[base:base + n]
            if bool(b.any()):
                off = int(torch.nonzero(b)[0])
                # the channel / round that carried it: swps_comm.hip ipc_span's split of an n-byte
                # segment into IPC_CHANNELS parts (16-B multiples, at least IPC_MIN_PART bytes),
                # each part streamed through sub-slots of slot / IPC_CHANNELS bytes
                part = max(IPC_MIN_PART, ((n + IPC_CHANNELS - 1) // IPC_CHANNELS + 15) & ~15)
                ch = off // part
                w0 = (base + off) & ~7
                report.append({"rank": rank, "peer": src, "channel": ch, "round": (off - ch * part) // sub,
                               "offset": off, "recv_offset": base + off, "segment_bytes": n,
                               "bad_bytes": int(b.sum()),
                               "expected": want[w0:w0 + 8].cpu().numpy().tobytes()[::-1].hex(),
                               "got": recv[w0:w0 + 8].cpu().numpy().tobytes()[::-1].hex()})
            base += n
        return False, report

    def set_timeout(self, seconds):
        """Deadline for the communicator's initialisation and each exchange (RCCL guard)."""
        check(capi.lib().swps_comm_set_timeout(self.h, float(seconds)))

    def check(self):
        """Raise SwpsError if the RCCL guard aborted this communicator."""
        check(capi.lib().swps_comm_check(self.h))

    def abort(self, why="aborted by the caller"):
        check(capi.lib().swps_comm_abort(self.h, why.encode()))

    def close(self):
        if getattr(self, "h", None):
            capi.lib().swps_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (AttributeError, TypeError):
            pass
