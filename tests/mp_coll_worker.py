"""A rank of tests/test_host_collectives_cpu.py: the host-transport callbacks
(crgc_hip.HostCollectives over gloo) called as the library calls them —
through their C function pointers, on pinned-memory-like ctypes buffers —
checked against the bytes every rank must receive.
usage: python tests/mp_coll_worker.py <rank> <world> <port>"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "uigc-akka_amd"))


def main():
    rank, n, port = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=n)
    import crgc_hip
    coll = crgc_hip.HostCollectives(n, rank)
    # all-gather: 13 bytes per rank
    nb = 13
    send = (C.c_uint8 * nb)(*[(rank * 31 + i) & 0xFF for i in range(nb)])
    recv = (C.c_uint8 * (nb * n))()
    assert coll.c.allgather(None, rank, C.addressof(send), C.addressof(recv), nb) == 0
    for r in range(n):
        assert list(recv[r * nb:(r + 1) * nb]) == [(r * 31 + i) & 0xFF for i in range(nb)], (r, list(recv))
    # all-to-all-v: rank s sends (s + 1) * (d + 2) bytes to d at 8-B-aligned offsets with gaps,
    # receives (r + 1) * (rank + 2) bytes from r
    size = lambda s, d: (s + 1) * (d + 2)  # noqa: E731
    soff, sb, so = [], [], 0
    for d in range(n):
        soff.append(so)
        sb.append(size(rank, d))
        so += (size(rank, d) + 7) // 8 * 8 + 8
    roff, rb, ro = [], [], 0
    for r in range(n):
        roff.append(ro)
        rb.append(size(r, rank))
        ro += size(r, rank) + 5
    sbuf = (C.c_uint8 * max(so, 1))()
    for d in range(n):
        for i in range(sb[d]):
            sbuf[soff[d] + i] = (rank * 7 + d * 13 + i) & 0xFF
    rbuf = (C.c_uint8 * max(ro, 1))()
    arr = lambda v: (C.c_size_t * n)(*v)  # noqa: E731
    assert coll.c.alltoallv(None, rank, C.addressof(sbuf), arr(soff), arr(sb), C.addressof(rbuf), arr(roff),
                            arr(rb)) == 0
    for r in range(n):
        got = list(rbuf[roff[r]:roff[r] + rb[r]])
        assert got == [(r * 7 + rank * 13 + i) & 0xFF for i in range(rb[r])], (r, got)
    # the library accepts the callbacks (no GPU work at creation)
    tr = crgc_hip.Transport.host(coll, device=0)
    tr.close()
    dist.barrier()
    dist.destroy_process_group()
    print("ok", rank)


if __name__ == "__main__":
    main()
