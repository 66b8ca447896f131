"""CPU-only checks of the drop-in boundary: libtrafficrl.so is built for
gfx950, loads, exports every symbol include/trafficrl.h declares, and the
ctypes struct layouts match the C header (checked by compiling the header
with gcc).  No compute call is made (no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT, golden

HEADER = os.path.join(ROOT, "include", "trafficrl.h")
LIB = os.path.join(PKG_DIR, "trafficrl", "libtrafficrl.so")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(trx_[a-z0-9_]+)\s*\(", txt)))


def test_library_exists_and_targets_gfx950():
    assert os.path.exists(LIB), "build with __graft_entry__.build()"
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob


def test_exports_every_declared_symbol():
    from trafficrl import _lib
    L = _lib.load()
    syms = declared_symbols()
    assert set(syms) == set(_lib.EXPORTS)
    for s in syms:
        assert hasattr(L, s), s
    assert L.trx_abi_version() == _lib.ABI_VERSION == 12


def test_struct_layout_matches_header(tmp_path):
    from trafficrl import _lib
    src = tmp_path / "probe.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "trafficrl.h"\n'
        "int main(){printf(\"%zu %zu %zu %zu %zu\\n\", sizeof(trx_params), offsetof(trx_params, unassigned_penalty),"
        " offsetof(trx_params, reward_alpha), offsetof(trx_params, reward_clip), sizeof(trx_state));return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    vals = list(map(int, subprocess.check_output([str(exe)]).split()))
    P = _lib.TrxParams
    assert vals == [ctypes.sizeof(P), P.unassigned_penalty.offset, P.reward_alpha.offset, P.reward_clip.offset,
                    ctypes.sizeof(_lib.TrxState)]


def test_error_path_without_gpu():
    """Graph creation reaches the HIP runtime; on a GPU-less host it must
    fail loudly (no silent CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from trafficrl.data import sioux_falls
    from trafficrl.graph import TrafficGraph
    with pytest.raises(RuntimeError):
        TrafficGraph(sioux_falls())


def test_tntp_parser_matches_reference_arrays():
    from trafficrl.data import sioux_falls
    z = np.load(golden("sf_graph.npz"))
    g = sioux_falls()
    assert g.num_nodes == int(z["num_nodes"])
    np.testing.assert_array_equal([e.u - 1 for e in g.edges], z["src"])
    np.testing.assert_array_equal([e.v - 1 for e in g.edges], z["dst"])
    np.testing.assert_array_equal(np.array([e.capacity for e in g.edges], np.float32), z["cap0"])
    np.testing.assert_array_equal(np.array([e.t0 for e in g.edges], np.float32), z["t0"])
    od = list(g.od_demand.items())
    np.testing.assert_array_equal([o - 1 for (o, _), _ in od], z["od_o"])
    np.testing.assert_array_equal([d - 1 for (_, d), _ in od], z["od_d"])
    np.testing.assert_array_equal([v for _, v in od], z["od_v"])


def test_damage_sampler_matches_reference_seeds():
    """Host damage draws == the reference's RepairEnv(seed=s).reset() sets."""
    from trafficrl.data import sioux_falls
    from trafficrl.graph import DamageSampler
    z = np.load(golden("sf_random_resets_crpow.npz"))
    g = sioux_falls()

    class G:  # the sampler only needs topology
        num_edges = len(g.edges)
        num_nodes = g.num_nodes
        src = np.array([e.u - 1 for e in g.edges], np.int32)
        dst = np.array([e.v - 1 for e in g.edges], np.int32)

    for i, s in enumerate(z["seeds"]):
        m = DamageSampler(G, int(s)).sample(0.3)
        np.testing.assert_array_equal(m, z["damaged"][i])
    fixed = DamageSampler(G, 0, fixed_damage=True, fixed_damage_seed=42).sample(0.3)
    r = np.load(golden("sf_reset_seed42_crpow.npz"))
    np.testing.assert_array_equal(fixed, r["msa30_damaged"])


def _reference_draw(rng, num_nodes, src, dst, ratio):
    """repair_env.py:167-192 restated with networkx (test-only checker)."""
    import networkx as nx
    E = len(src)
    G = nx.DiGraph()
    for i, (u, v) in enumerate(zip(src.tolist(), dst.tolist())):
        G.add_edge(u, v, edge_id=i)
    count = max(1, int(E * ratio))
    for _ in range(50):
        cand = rng.choice(E, size=count, replace=False)
        m = np.zeros(E, np.float32)
        m[cand] = 1.0
        active = [(u, v) for u, v, d in G.edges(data=True) if m[d["edge_id"]] == 0]
        if not active:
            continue
        if nx.is_strongly_connected(G.edge_subgraph(active).copy()):
            return m
    m = np.zeros(E, np.float32)
    m[rng.choice(E, size=count, replace=False)] = 1.0
    return m


@pytest.mark.parametrize("net", ["sf", "ana", "parallel"])
def test_batch_damage_sampler_matches_numpy_generator(net):
    """trx_damage_sample (numpy's PCG64 + choice restated natively) == the
    reference's loop on numpy Generators: masks over 3 successive resets per
    env, and the generator states afterwards (so later draws stay in step).
    'parallel' adds a duplicate (u, v) link: the DiGraph keeps the last id."""
    from trafficrl.graph import damage_sample_batch, pcg_states, set_generator_state
    if net == "sf":
        from trafficrl.data import sioux_falls
        g = sioux_falls()
        src = np.array([e.u - 1 for e in g.edges], np.int32)
        dst = np.array([e.v - 1 for e in g.edges], np.int32)
        N, envs, ratios = g.num_nodes, 64, (0.3, 0.1, 0.5)
    elif net == "ana":
        z = np.load(golden("ana_graph.npz"))
        src, dst, N, envs, ratios = z["src"].astype(np.int32), z["dst"].astype(np.int32), int(z["num_nodes"]), 6, \
            (0.3, 0.05, 0.3)
    else:
        rng = np.random.default_rng(3)
        N = 8
        ring = [(i, (i + 1) % N) for i in range(N)] + [((i + 1) % N, i) for i in range(N)]
        extra = [tuple(map(int, rng.integers(0, N, 2))) for _ in range(10)]
        pairs = ring + extra + ring[:4]     # ring[:4] again: parallel links
        src = np.array([p[0] for p in pairs], np.int32)
        dst = np.array([p[1] for p in pairs], np.int32)
        envs, ratios = 40, (0.3, 0.2, 0.4)
    seeds = [1000 + i for i in range(envs)]
    gens = [np.random.default_rng(s) for s in seeds]
    st = pcg_states(seeds)
    for ratio in ratios:
        got = damage_sample_batch(N, src, dst, st, ratio, nthreads=3)
        want = np.stack([_reference_draw(r, N, src, dst, ratio) for r in gens])
        np.testing.assert_array_equal(got, want)
    for r, rec in zip(gens, st):
        probe = np.random.default_rng(0)
        set_generator_state(probe, rec)
        assert probe.bit_generator.state == r.bit_generator.state
        assert probe.random() == r.random()


def test_fused_args_layout_matches_header(tmp_path):
    """Every field offset of the fused kernels' argument structs (incl. ABI
    10's exact fields, the round list's dst_stride, trx_psum_list and ABI 11's
    trx_edge_head_bwd_io) as the C
    compiler lays them out equals the ctypes mirror in trafficrl/_lib.py."""
    from trafficrl import _lib
    lines = []
    structs = (("trx_gat_layer_args", _lib.TrxGatLayerArgs), ("trx_edge_head_args", _lib.TrxEdgeHeadArgs),
               ("trx_gat_prologue_args", _lib.TrxGatPrologueArgs), ("trx_gat_layer0_args", _lib.TrxGatLayer0Args),
               ("trx_gat_mid_args", _lib.TrxGatMidArgs), ("trx_gat_layer_bwd_args", _lib.TrxGatLayerBwdArgs),
               ("trx_gat_prologue_bwd_args", _lib.TrxGatPrologueBwdArgs), ("trx_round_list", _lib.TrxRoundList),
               ("trx_psum_list", _lib.TrxPsumList), ("trx_edge_head_bwd_io", _lib.TrxEdgeHeadBwdIO))
    for cname, cls in structs:
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("%zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "probe2.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"trafficrl.h\"\nint main(){" + "".join(lines)
                   + "return 0;}\n")
    exe = tmp_path / "probe2"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    vals = list(map(int, subprocess.check_output([str(exe)]).split()))
    want = []
    for _, cls in structs:
        want.append(ctypes.sizeof(cls))
        want += [getattr(cls, f).offset for f, _ in cls._fields_]
    assert vals == want


def test_round_and_psum_lists_validated_without_gpu():
    """trx_bf16_round (modes 0-3, dst_stride) and trx_partial_sum_multi refuse
    malformed lists before any HIP call; empty lists are no-ops."""
    from trafficrl import _lib
    L = _lib.load()
    lst = _lib.TrxRoundList()
    lst.count = 1
    lst.rows[0], lst.cols[0], lst.src_stride[0] = 2, 8, 8
    lst.src[0], lst.dst[0] = 16, 16          # never dereferenced: refused first
    lst.out_bf16[0] = 4
    assert L.trx_bf16_round(ctypes.byref(lst), None) == -1
    lst.out_bf16[0], lst.dst_stride[0] = 3, 4  # dst rows narrower than the block
    assert L.trx_bf16_round(ctypes.byref(lst), None) == -1
    lst.count = 0
    assert L.trx_bf16_round(ctypes.byref(lst), None) == 0
    ps = _lib.TrxPsumList()
    ps.count = _lib.MAX_PSUM + 1
    assert L.trx_partial_sum_multi(ctypes.byref(ps), None) == -1
    ps.count, ps.rows = 1, 4
    ps.part[0], ps.out[0], ps.width[0], ps.stride[0] = 16, 16, 8, 4   # stride < width
    assert L.trx_partial_sum_multi(ctypes.byref(ps), None) == -1
    ps.count = 0
    assert L.trx_partial_sum_multi(ctypes.byref(ps), None) == 0


def test_weighted_sample_validated_without_gpu():
    """trx_per32_sample_weighted refuses missing buffers / a bad capacity before
    any HIP call; an empty batch is a no-op."""
    from trafficrl import _lib
    L = _lib.load()
    f = L.trx_per32_sample_weighted
    assert f(None, 8, 16, 4, 16, 0.4, 16, 16, 16, None) == -1          # no tree
    assert f(16, 0, 16, 4, 16, 0.4, 16, 16, 16, None) == -1            # capacity < 1
    assert f(16, 8, 16, 4, None, 0.4, 16, 16, 16, None) == -1          # no size
    assert f(16, 8, 16, 4, 16, 0.4, 16, 16, None, None) == -1          # no weight output
    assert f(16, 8, 16, -1, 16, 0.4, 16, 16, 16, None) == -1           # n < 0
    assert f(16, 8, None, 0, None, 0.4, None, None, None, None) == 0   # empty batch


def test_fused_infer_validation_without_gpu():
    """Argument checks run before any HIP call: unsupported shapes are refused
    with TRX_EUNSUP / TRX_EINVAL and a message."""
    from trafficrl import _lib
    L = _lib.load()
    a = _lib.TrxGatLayerArgs()
    a.num_graphs, a.nodes_per_graph, a.heads, a.channels, a.concat, a.max_graph_edges = 4, 64, 4, 256, 1, 100
    assert L.trx_gat_layer_infer(a, None) == -3
    assert b"nodes_per_graph" in L.trx_last_error()
    a.nodes_per_graph = 24
    assert L.trx_gat_layer_infer(a, None) == -1       # NULL layer input
    h = _lib.TrxEdgeHeadArgs()
    h.num_graphs, h.edges_per_graph, h.hidden, h.edge_dim = 4, 76, 256, 32
    assert L.trx_edge_head_infer(h, None) == -3
    pa = _lib.TrxGatPrologueArgs()
    pa.num_graphs, pa.nodes_per_graph, pa.edges_per_graph, pa.node_dim, pa.edge_dim = 4, 24, 76, 4, 6
    pa.num_layers = 5
    assert L.trx_gat_prologue_infer(pa, None) == -3
    assert b"num_layers" in L.trx_last_error()
    pa.num_layers, pa.heads[0], pa.channels[0] = 1, 4, 256
    assert L.trx_gat_prologue_infer(pa, None) == -1    # NULL weights
    h.edge_dim, h.nodes_per_graph = 6, 200             # p rows of one graph would not fit in LDS
    assert L.trx_edge_head_infer(h, None) == -3
    assert b"nodes_per_graph" in L.trx_last_error()


def test_no_packed_fp32_instructions(tmp_path):
    """The library is built without packed-FP32 VALU instructions (Makefile
    -target-feature -packed-fp32-ops): on gfx950 their results can reach a DPP
    or packed consumer two wait states later without the last 16 lanes while
    another kernel's waves share the CU -- the round-4 nondeterminism of the
    concurrently replayed SAC update (tests/test_concurrent_update.py)."""
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    from trafficrl import codeobj
    cos = codeobj._code_objects(open(LIB, "rb").read())
    assert cos, "no gfx950 code objects in the library"
    hits = {}
    for k, co in enumerate(cos):
        path = tmp_path / f"co{k}.o"
        path.write_bytes(co)
        asm = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(path)], check=True, capture_output=True,
                             text=True).stdout
        n = len(re.findall(r"\bv_pk_(?:add|mul|fma)_f32\b", asm))
        assert "s_endpgm" in asm
        if n:
            hits[k] = n
    assert not hits, f"packed-FP32 instructions in code objects {hits}"


def test_integration_snippet_matches_abi():
    """INTEGRATION.md §2's reference-side ctypes binding stays in step with the
    header: its ABI assertion is the library's version and its TrxParams /
    TrxState fields have the layouts of trafficrl._lib's (checked against the
    header by test_struct_layout_matches_header)."""
    import ctypes as C
    from trafficrl import _lib
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"trx_abi_version\(\) == (\d+)", doc)
    assert m and int(m.group(1)) == _lib.ABI_VERSION == ctypes.CDLL(LIB).trx_abi_version()
    code = doc[doc.index("class TrxParams"):doc.index("g = ctypes.c_void_p()")]
    ns = {"ctypes": C}
    exec(code, ns)   # the two Structure definitions of the snippet
    for name, ref in (("TrxParams", _lib.TrxParams), ("TrxState", _lib.TrxState)):
        mine = ns[name]
        assert C.sizeof(mine) == C.sizeof(ref), name
        assert [(f[0], getattr(mine, f[0]).offset) for f in mine._fields_ if not f[0].startswith("_")] == \
               [(f[0], getattr(ref, f[0]).offset) for f in ref._fields_ if not f[0].startswith("_")], name


def test_multi_launches_validated_without_gpu():
    """The *_multi entry points (ABI 11) refuse a network count outside
    1..TRX_MAX_NETS and networks whose shapes differ, before any HIP call."""
    from trafficrl import _lib
    L = _lib.load()
    a = _lib.TrxGatLayerArgs()
    assert L.trx_gat_layer_infer_multi(_lib.multi(_lib.TrxGatLayerArgs, [a]), 0, None) == _lib.TRX_EINVAL
    assert L.trx_gat_layer_infer_multi(_lib.multi(_lib.TrxGatLayerArgs, [a] * 7), 7, None) == _lib.TRX_EINVAL
    # two otherwise valid blocks that differ in heads: refused as a pair
    keep = []
    def block(heads):
        b = _lib.TrxGatLayerArgs()
        b.num_graphs, b.nodes_per_graph, b.heads, b.channels, b.concat, b.max_graph_edges = 0, 24, heads, 256 // heads, 1, 100
        b.in_dim, b.residual, b.activation = 0, 0, 0
        buf = (ctypes.c_float * 16)()
        keep.append(buf)
        p = ctypes.addressof(buf)
        b.xh = b.rowptr = b.col = b.a_edge = b.att_src = b.att_dst = b.bias = b.ln_weight = b.ln_bias = p
        b.out_bf16 = p
        b.a_edge_stride, b.a_edge_offset = 8, 0
        return b
    assert L.trx_gat_layer_infer_multi(_lib.multi(_lib.TrxGatLayerArgs, [block(4), block(4)]), 2, None) == 0
    rc = L.trx_gat_layer_infer_multi(_lib.multi(_lib.TrxGatLayerArgs, [block(4), block(2)]), 2, None)
    assert rc == _lib.TRX_EINVAL and b"differs" in L.trx_last_error()
    io = _lib.TrxEdgeHeadBwdIO()
    assert L.trx_edge_head_backward_multi(_lib.multi(_lib.TrxEdgeHeadArgs, [_lib.TrxEdgeHeadArgs()]),
                                          _lib.multi(_lib.TrxEdgeHeadBwdIO, [io]), 0, None) == _lib.TRX_EINVAL
    # the backward's networks must agree like the forward's, and on the presence of grad_z
    def eh(softmax, gz):
        b = _lib.TrxEdgeHeadArgs()
        b.num_graphs, b.edges_per_graph, b.nodes_per_graph, b.hidden, b.edge_dim, b.softmax = 0, 76, 24, 256, 6, softmax
        buf = (ctypes.c_float * 16)()
        keep.append(buf)
        p = ctypes.addressof(buf)
        b.src = b.dst = b.p = b.c = b.ea = b.we = b.w2 = p
        o = _lib.TrxEdgeHeadBwdIO()
        o.grad_logits = o.grad_p = o.grad_c = o.grad_w2_part = o.grad_we_part = o.grad_ea = p
        o.grad_z = p if gz else None
        return b, o
    def bwd(*nets):
        return L.trx_edge_head_backward_multi(_lib.multi(_lib.TrxEdgeHeadArgs, [n[0] for n in nets]),
                                              _lib.multi(_lib.TrxEdgeHeadBwdIO, [n[1] for n in nets]), len(nets), None)
    assert bwd(eh(0, False), eh(0, False)) == 0
    assert bwd(eh(0, False), eh(1, False)) == _lib.TRX_EINVAL
    assert bwd(eh(0, True), eh(0, False)) == _lib.TRX_EINVAL and b"differs" in L.trx_last_error()
