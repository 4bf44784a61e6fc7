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
    q_addr.put((rank, (server.address, os.getpid())))
    peers = addrs.get()                       # every rank's address, once all have served
    server.allow(pid for r, (_, pid) in peers.items() if r != rank)
    peers = {r: a for r, (a, _) in peers.items()}
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
    addrs = dict(q_addr.get(timeout=180) for _ in range(world))
    for q in addr_qs:
        q.put(addrs)
    out = dict(results.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    for rank, got in out.items():
        for r, contents in got.items():
            assert contents == ["rank%d-chunk%d" % (r, c) for c in range(chunks)], (rank, r)


def _intruder(address, q):
    from dpwa_amd.group import _fetch_fds
    try:
        _fetch_fds(address, 2)
        q.put("got fds")
    except Exception as e:   # noqa: BLE001
        q.put("refused: %s" % type(e).__name__)


def test_fds_are_served_only_to_the_ranks():
    """A process that is not one of the job's ranks (another pid) connects first: it gets no
    fds, and the rank that connects after it is still served (advisor finding on _FdServer)."""
    from dpwa_amd.group import _FdServer, _fetch_fds
    fds = [os.memfd_create("c%d" % c) for c in range(2)]
    for c, fd in enumerate(fds):
        os.write(fd, b"chunk%d" % c)
    server = _FdServer(fds, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_intruder, args=(server.address, q))
    p.start()
    server.allow([os.getpid()])             # this process stands for the peer rank
    assert q.get(timeout=60).startswith("refused")
    p.join(30)
    got = _fetch_fds(server.address, 2)
    assert [os.pread(fd, 16, 0) for fd in got] == [b"chunk0", b"chunk1"]
    for fd in got:
        os.close(fd)
    server.finish()
    assert server.rejected == 1


def test_abort_stops_serving_at_once():
    """An exchange that failed elsewhere (on_bind's collective raised): abort() ends the serving
    thread immediately instead of leaving it in accept() for TIMEOUT_S."""
    import time
    from dpwa_amd.group import _FdServer, _fetch_fds
    fd = os.memfd_create("c")
    server = _FdServer([fd], 2)
    t0 = time.monotonic()
    server.abort()
    server.thread.join(5)
    assert not server.thread.is_alive() and time.monotonic() - t0 < 5
    try:
        _fetch_fds(server.address, 1)
        raise AssertionError("an aborted server handed out fds")
    except OSError:
        pass
    os.close(fd)
