"""Host-side decisions of the custom P2P all-reduce (parallel/custom_ar.py) that need no GPU."""
from llm_map_reduce_summarizer_amd.parallel.custom_ar import CustomAllReduce, graph_safe

ONE, ROWS = CustomAllReduce.ONE_SHOT_MAX, CustomAllReduce.MAX_ROWS


def _paths(**kw):
    p = {k: True for k in CustomAllReduce.PATHS}
    p.update(kw)
    return p


def test_graph_safe_needs_the_key_max():
    assert not graph_safe(_paths(max_u64=False), 4096, ONE, ROWS)


def test_graph_safe_with_the_fused_path():
    assert graph_safe(_paths(one_shot=False), 4096, ONE, ROWS)
    assert graph_safe(_paths(one_shot=False), 8192, ONE, ROWS)


def test_fused_path_failed_one_shot_does_not_cover_every_bucket():
    # with fused_norm off, decode reduces one fp32 slab [M, hidden] on the one-shot kernel; at
    # hidden 4096 that fits 64 rows, not the 256-row bucket, so the handle is not graph-safe
    assert not graph_safe(_paths(fused_norm=False), 4096, ONE, ROWS)
    assert not graph_safe(_paths(fused_norm=False), 8192, ONE, ROWS)
    # ... unless the largest bucket's slab fits
    assert graph_safe(_paths(fused_norm=False), 4096, ONE, 64)
    assert not graph_safe(_paths(fused_norm=False, one_shot=False), 4096, ONE, 16)


def test_async_works_drops_waited_handles():
    """a waited handle leaves the scope at once (RCCL's WorkNCCL pins its outputs while alive);
    only pending handles are waited on exit, including on the exception path."""
    from llm_map_reduce_summarizer_amd.parallel.dist import AsyncWorks

    class W:
        def __init__(self):
            self.waits = 0

        def wait(self):
            self.waits += 1

    a, b = W(), W()
    with AsyncWorks() as works:
        works.add(a)
        works.add(b)
        works.add(None)
        assert len(works) == 2
        works.wait(a)
        works.wait(None)
        assert len(works) == 1
    assert a.waits == 1 and b.waits == 1
    c = W()
    try:
        with AsyncWorks() as works:
            works.add(c)
            raise KeyError("boom")
    except KeyError:
        pass
    assert c.waits == 1
