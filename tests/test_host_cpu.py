"""CPU: host-side logic of the product package (no GPU compute): parameter layout vs the reference
state-dict, RoPE tables vs the oracle, tokenizer, optimizer schedule, C-ABI symbol export."""

import ctypes
import math
import os
import re

import pytest
import torch

from oracle import jit_oracle as O
from tests.golden import golden_configs as GC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def vcfg(oc):
    from vpt.config import DenoiserConfig
    return DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                          bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                          context_start_block=oc.context_start_block)


@pytest.mark.parametrize("oc", [O.jit_b16(), GC.micro_config(), GC.c1_config()])
def test_param_layout_matches_reference_state_dict(oc):
    from vpt.params import ParamLayout
    lay = ParamLayout(vcfg(oc), n_classes=10)
    ref = {k: tuple(v.shape) for k, v in O.OracleJiT(oc).state_dict().items()}
    ref["class_encoder.embedding.weight"] = (11, oc.context_dim)
    got = {s.name: tuple(s.shape) for s in lay.specs}
    assert got == ref
    # no overlaps, fused groups adjacent
    spans = sorted((s.offset, s.offset + s.numel, s.name) for s in lay.specs)
    for (a0, a1, an), (b0, b1, bn) in zip(spans, spans[1:]):
        assert a1 <= b0, (an, bn)
    for i in range(oc.depth):
        p = f"blocks.{i}."
        q, k, v = (lay.by_name[p + f"attn.to_{x}.weight"] for x in "qkv")
        assert k.offset == q.offset + q.numel and v.offset == k.offset + k.numel
        w1, w2 = lay.by_name[p + "mlp.w_1.weight"], lay.by_name[p + "mlp.w_2.weight"]
        assert w2.offset == w1.offset + w1.numel
        qn, kn = lay.by_name[p + "attn.q_norm.weight"], lay.by_name[p + "attn.k_norm.weight"]
        assert kn.offset == qn.offset + qn.numel
    assert lay.total >= sum(s.numel for s in lay.specs)


def test_jit_b16_param_count():
    from vpt.config import JiT_B_16_Config
    from vpt.params import ParamLayout
    lay = ParamLayout(JiT_B_16_Config())
    assert sum(s.numel for s in lay.specs) == 92_731_648  # SURVEY Appendix A, verified on the reference


@pytest.mark.parametrize("hw", [(16, 16), (64, 64), (60, 68), (56, 72), (4, 3)])
def test_rope_angles_match_oracle(hw):
    from vpt.config import JiT_B_16_Config
    from vpt.rope import rope_angles
    hp, wp = hw
    ang = rope_angles(JiT_B_16_Config(), hp, wp, 64)
    fc = O.rope_freqs(O.jit_b16(), hp, wp, 64)
    c = torch.polar(torch.ones_like(ang), ang)
    assert torch.equal(c, fc)


def test_rope_rejects_oversize_bucket():
    from vpt.config import JiT_B_16_Config
    from vpt.rope import rope_angles
    with pytest.raises(ValueError):
        rope_angles(JiT_B_16_Config(), 2368 // 16, 448 // 16, 64)


def test_tokenizer_matches_oracle():
    from vpt.jit_train import ClassTokenizer
    l2i = {f"c{i}": i for i in range(7)}
    caps = ["c1 c2", "", "c6 nope c0", "c1 " * 20]
    tok = ClassTokenizer(l2i)
    with pytest.warns(UserWarning):
        ids, mask = tok.tokenize(caps, 8)
    rid, rmask = O.class_tokenize(caps, l2i, 8)
    assert torch.equal(ids, rid) and torch.equal(mask, rmask)


def test_radam_sf_scalar_schedule():
    """vpt.optim's host schedule == the published schedulefree step (tests/sf_reference.py), incl.
    weight = step**r * lr_max**weight_lr_power with r = 0 (1/k-like averaging, not 3/k)."""
    import vpt.optim as vo
    from tests.sf_reference import reference_schedule
    for r, wlp, silent in ((0.0, 2.0, True), (0.5, 1.0, False)):
        opt = vo.RAdamScheduleFreeFlat.__new__(vo.RAdamScheduleFreeFlat)
        opt.param_groups = [dict(lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, r=r, k=0, train_mode=True,
                                 weight_sum=0.0, lr_max=-1.0, scheduled_lr=0.0, weight_lr_power=wlp,
                                 silent_sgd_phase=silent)]
        ref = reference_schedule(1e-4, (0.9, 0.999), 40, r=r, weight_lr_power=wlp, silent_sgd_phase=silent)
        for k in range(40):
            s = opt.scalars()
            g = opt.param_groups[0]
            assert math.isclose(s["lr"], ref[k][0], rel_tol=1e-12, abs_tol=1e-20)
            assert math.isclose(s["ckp1"], ref[k][1], rel_tol=1e-12, abs_tol=1e-20)
            assert s["adam"] == ref[k][2]
            g["lr_max"], g["weight_sum"], g["k"] = s["lr_max"], s["weight_sum"], g["k"] + 1
        if silent:
            assert ref[0][0] == 0.0 and ref[0][1] == 0.0 and ref[-1][0] > 0  # silent SGD warm-up, then RAdam
        else:
            assert ref[0][0] == 1e-4  # plain SGD at the full lr during the warm-up
    # r = 0: averaging weight -> 1/k once the rectified lr has settled (the r1 build's step**p gave ~3/k)
    sch = reference_schedule(1e-3, (0.9, 0.999), 20000)
    assert 0.9 < sch[-1][1] * 20000 < 1.2


def test_radam_sf_restatement_matches_closed_form():
    """The CPU restatement used as the GPU kernel's checker reproduces the closed form of one
    Adam-phase step on a scalar (guards the checker itself)."""
    from tests.sf_reference import SFRef
    y = torch.tensor([0.5], dtype=torch.float32)
    opt = SFRef([y], lr=1e-2, weight_decay=0.1, silent_sgd_phase=False)
    opt.train()
    g = torch.tensor([0.2])
    s = opt.step([g])  # step 1: rho_t <= 4, silent_sgd_phase False -> plain SGD at lr
    assert s["rho_t"] <= 4 and s["ckp1"] == 1.0
    gd = 0.2 + 0.1 * 0.5
    assert math.isclose(opt.z[0].item(), 0.5 - 1e-2 * gd, rel_tol=1e-6)
    assert math.isclose(y.item(), 0.5 + (1e-2 * (0.9 * 0 - 1)) * gd, rel_tol=1e-6)


def test_capi_exports_every_declared_symbol():
    """include/vpt_hip.h declarations == symbols exported by libvpt_hip.so == Python bindings."""
    from vpt import _lib
    hdr = open(os.path.join(ROOT, "include", "vpt_hip.h")).read()
    declared = set(re.findall(r"\b(vpt_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(_lib.SIGNATURES), (declared ^ set(_lib.SIGNATURES))
    # the production library is stateless: no process-wide A/B or ablation switch is exported
    # (those live only in libvpt_hip_diag.so, include/vpt_hip_diag.h)
    diag = set(re.findall(r"\b(vpt_[a-z0-9_]+)\s*\(", open(os.path.join(ROOT, "include", "vpt_hip_diag.h")).read()))
    assert diag == set(_lib.DIAG_SIGNATURES)
    leaked = [s for s in diag if hasattr(ctypes.CDLL(str(_lib.LIB)), s)]
    assert not leaked, leaked


def test_capi_reports_errors_without_gpu_work():
    """Argument validation happens before any launch: a bad shape returns VPT_EINVAL + message."""
    from vpt import _lib
    rc = _lib.lib.vpt_gemm_bf16(None, 0, 1, None, 0, 1, None, 0, 0, 0, 0, None, None, 0, 0, 0, 1, None, 1.0, None)
    assert rc == 1
    assert b"null operand" in _lib.lib.vpt_last_error_string()


def test_sub_pool_slices_one_storage():
    """engine._SubPool (the sub-batch lanes' view of the buffer pool): lane h of n gets rows [h*r, (h+1)*r) of ONE
    pooled buffer of n*r rows, whatever the trailing shape, so the lanes write disjoint halves the one-lane backward
    then reads whole."""
    import torch

    from vpt.engine import _Pool, _SubPool
    pool = _Pool(torch.device("cpu"))
    a, b = _SubPool(pool, 0, 2).get("x", (3, 4)), _SubPool(pool, 1, 2).get("x", (3, 4))
    full = pool.get("x", (6, 4))
    a.fill_(1.0)
    b.fill_(2.0)
    assert full[:3].eq(1.0).all() and full[3:].eq(2.0).all()
    lse0 = _SubPool(pool, 0, 2).get("lse", (2, 5, 7), torch.float32)
    lse1 = _SubPool(pool, 1, 2).get("lse", (2, 5, 7), torch.float32)
    whole = pool.get("lse", (4, 5, 7), torch.float32)
    assert lse0.data_ptr() == whole.data_ptr() and lse1.data_ptr() == whole[2:].data_ptr()
    assert lse1.shape == (2, 5, 7)
