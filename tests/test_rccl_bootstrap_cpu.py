"""``RcclComm``'s multi-rank bootstrap (``parallel/rccl.py``) on 4 gloo ranks with the RCCL library mocked: the code
path the first multi-GPU ``--transport rccl`` run takes before any ``ncclCommInitRank`` - namespaces, store keys,
per-edge unique ids, init order and comm-local peer indices."""
import json
import socket

import torch.multiprocessing as mp

import dist_worker


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_bootstrap_four_rank_chain(tmp_path):
    world = 4
    out = tmp_path / "boot"
    mp.spawn(dist_worker.run_rccl_bootstrap, args=(world, _port(), str(out)), nprocs=world, join=True)
    rep = [json.loads((tmp_path / f"boot.{r}").read_text()) for r in range(world)]
    for c in range(2):                                       # two constructions in a row
        gens = {rep[r][c]["gen"] for r in range(world)}
        assert len(gens) == 1, gens                          # one namespace, broadcast from rank 0
    assert rep[0][0]["gen"] != rep[0][1]["gen"]              # fresh namespace per construction
    for c in range(2):
        for r in range(world):
            x = rep[r][c]
            want = [[a, a + 1] for a in (r - 1, r) if 0 <= a and a + 1 < world]
            assert x["channels"] == want                     # one channel per pipeline edge, global sorted init order
            assert [i["nranks"] for i in x["inits"]] == [2] * len(want)
            for (a, b), init in zip(x["channels"], x["inits"]):
                assert init["idx"] == (0 if r == a else 1)   # comm-local rank: lower pipeline rank is 0
                assert init["device"] == r % 8
                assert init["uid"].startswith(f"uid-made-by-{a}-")   # the edge's lower rank made its id
            for p, i in x["peer_index"].items():
                assert i == (0 if int(p) < r else 1)
            assert x["keys_left"] == []                      # the reader deleted each id key
            assert set(x["h"]) <= set(x["destroyed"])       # close() destroyed every communicator
        # both ends of an edge initialised with the same id
        for a in range(world - 1):
            ua = [i["uid"] for i, ch in zip(rep[a][c]["inits"], rep[a][c]["channels"]) if ch == [a, a + 1]]
            ub = [i["uid"] for i, ch in zip(rep[a + 1][c]["inits"], rep[a + 1][c]["channels"]) if ch == [a, a + 1]]
            assert ua == ub and len(ua) == 1
    # ids are never reused across constructions
    assert rep[0][0]["inits"][0]["uid"] != rep[0][1]["inits"][0]["uid"]
