"""a26 host logic: vpt.trainer.SavingStrategy vs the reference's ModelSavingStrategy decisions and checks,
and the checkpoint file-name template incl. the EMA prefix (tests/golden/saving.safetensors, generated
from src/saving/util.py by tests/golden/make_golden.py saving)."""
import json
import os
import sys

import pytest
from safetensors import safe_open

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

from vpt.trainer import SafetensorsSaver, SavingStrategy  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "saving.safetensors")


def _fx():
    with safe_open(GOLD, "pt") as f:
        md = f.metadata()
        return {k: f.get_tensor(k) for k in f.keys()}, md


def test_should_save_matches_reference():
    fx, md = _fx()
    cases = json.loads(md["cases"])
    for ci, c in enumerate(cases):
        st = SavingStrategy(**c)
        for epoch, step, want in fx[f"case{ci}"].tolist():
            assert st.should_save(epoch, step) == bool(want), (c, epoch, step)


def test_invalid_strategies_raise_like_reference():
    fx, md = _fx()
    for c, r in zip(json.loads(md["bad"]), fx["bad_raises"].tolist()):
        if r:
            with pytest.raises(ValueError):
                SavingStrategy(**c)
        else:
            SavingStrategy(**c)


def test_file_names_and_ema_prefix(tmp_path):
    _, md = _fx()
    assert SafetensorsSaver.template == md["template"]
    names = json.loads(md["names"])
    s = SafetensorsSaver("jit", str(tmp_path))
    assert [s.template.format(name="jit", epoch=e, steps=n) for e, n in ((1, 10), (12, 123456))] == names
    e = SafetensorsSaver("jit", str(tmp_path), "ema_" + s.template)
    assert e.template.format(name="jit", epoch=1, steps=10) == "ema_" + names[0]
