"""CPU: the fd hand-over DistGroup uses for snapshot allocations of 1.5 GiB and more
(group.py _FdServer / _fetch_fds): every rank serves its chunk fds to each peer over an
abstract Unix socket (SCM_RIGHTS) and fetches every peer's; memfds stand in for the
hipMemCreate chunks, and each receiver reads through the received fds what the owner wrote."""
import multiprocessing as mp
import os


def _rank(rank, world, q_addr, addrs, results, chunks):
    from dpwa_amd.group import _FdServer, _fetch_fds
    fds = []
    for c in range(chunks):
        fd = os.memfd_create("chunk%d" % c)
        os.write(fd, b"rank%d-chunk%d" % (rank, c))
        fds.append(fd)
    server = _FdServer(fds, world - 1)
    q_addr.put((rank, server.address))
    peers = addrs.get()                       # every rank's address, once all have served
    got = {}
    for r in range(world):
        if r == rank:
            continue
        rfds = _fetch_fds(peers[r], chunks)
        got[r] = []
        for fd in rfds:
            os.lseek(fd, 0, os.SEEK_SET)
            got[r].append(os.read(fd, 64).decode())
            os.close(fd)
    server.finish()
    results.put((rank, got))


def test_fds_reach_every_peer():
    world, chunks = 3, 4
    ctx = mp.get_context("spawn")
    q_addr, results = ctx.Queue(), ctx.Queue()
    addr_qs = [ctx.Queue() for _ in range(world)]
    ps = [ctx.Process(target=_rank, args=(r, world, q_addr, addr_qs[r], results, chunks)) for r in range(world)]
    for p in ps:
        p.start()
    addrs = dict(q_addr.get(timeout=60) for _ in range(world))
    for q in addr_qs:
        q.put(addrs)
    out = dict(results.get(timeout=60) for _ in range(world))
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for rank, got in out.items():
        for r, contents in got.items():
            assert contents == ["rank%d-chunk%d" % (r, c) for c in range(chunks)], (rank, r)
