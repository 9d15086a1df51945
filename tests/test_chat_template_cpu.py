"""Chat-template parity (reference D3/I1/I2: ``apply_chat_template`` with the tokenizer's own template,
``training.py:282-283``, ``ask_tuned_model.py:45-49``, ``enable_thinking=False`` at
``ask_original_model.py:44``). The Jinja path renders a template shipped with the tokenizer; the built-in
renderer is the offline fallback. Both are pinned against a fixture template shaped like SmolLM3's hub
template (the hub file itself is not available offline: parity with it stays unpinned)."""
import json
import os
import tempfile

import pytest

from llm_fine_tune_distributed_amd.data import chat_template as ct
from llm_fine_tune_distributed_amd.data.prompts import WILDERNESS_EXPERT_SYSTEM_PROMPT, format_prompt
from llm_fine_tune_distributed_amd.data.tokenizer import load_tokenizer

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "smollm3_like_chat_template.jinja")
ROWS = [{"full-question": "For Essential Knots and Uses, how do I tie a bowline?", "answer": "Form a loop, pass..."},
        {"full-question": "For Common Unit Conversions, what is 1 mile in km?", "answer": "About 1.609 km — ünïcode ok."}]


@pytest.fixture(scope="module")
def tpl():
    return open(FIX).read()


@pytest.fixture(scope="module")
def tok():
    return load_tokenizer(corpus=[r["full-question"] for r in ROWS] + [r["answer"] for r in ROWS])


@pytest.mark.parametrize("gen", [False, True])
@pytest.mark.parametrize("thinking", [False, True])
def test_jinja_fixture_matches_builtin_renderer(tpl, gen, thinking):
    for r in ROWS:
        msgs = format_prompt(r)["messages"]
        if gen:
            msgs = msgs[:-1]
        a = ct.render_jinja(tpl, msgs, add_generation_prompt=gen, enable_thinking=thinking)
        b = ct.render(msgs, add_generation_prompt=gen, enable_thinking=thinking)
        assert a == b


def test_tokenizer_uses_its_own_template_when_present(tok, tpl):
    d = tempfile.mkdtemp()
    tok.save_pretrained(d)
    cfg = json.load(open(os.path.join(d, "tokenizer_config.json")))
    marker = "{{ '<<JINJA>>' }}" + tpl
    cfg["chat_template"] = marker
    json.dump(cfg, open(os.path.join(d, "tokenizer_config.json"), "w"))
    t2 = load_tokenizer(d)
    msgs = format_prompt(ROWS[0])["messages"]
    text = t2.apply_chat_template(msgs, tokenize=False)
    assert text.startswith("<<JINJA>>") and text[len("<<JINJA>>"):] == ct.render(msgs)
    # a list of named templates (HF format) selects "default"; a chat_template.jinja file is picked up too
    cfg["chat_template"] = [{"name": "tool_use", "template": "x"}, {"name": "default", "template": marker}]
    json.dump(cfg, open(os.path.join(d, "tokenizer_config.json"), "w"))
    assert load_tokenizer(d).apply_chat_template(msgs, tokenize=False) == text
    del cfg["chat_template"]
    json.dump(cfg, open(os.path.join(d, "tokenizer_config.json"), "w"))
    open(os.path.join(d, "chat_template.jinja"), "w").write(marker)
    t3 = load_tokenizer(d)
    assert t3.apply_chat_template(msgs, tokenize=False) == text
    # enable_thinking reaches the template (ask_original_model.py:44)
    gp = t3.apply_chat_template(msgs[:-1], tokenize=False, add_generation_prompt=True, enable_thinking=False)
    assert gp.endswith("<|im_start|>assistant\n<think>\n\n</think>\n") and "/no_think" in gp
    gp = t3.apply_chat_template(msgs[:-1], tokenize=False, add_generation_prompt=True, enable_thinking=True)
    assert gp.endswith("<|im_start|>assistant\n") and "/think" in gp
    # the saved tokenizer keeps its template
    d2 = tempfile.mkdtemp()
    t3.save_pretrained(d2)
    assert load_tokenizer(d2).chat_template == marker


def test_builtin_fallback_when_no_template(tok):
    assert tok.chat_template is None
    msgs = format_prompt(ROWS[1])["messages"]
    assert tok.apply_chat_template(msgs, tokenize=False) == ct.render(msgs)
    ids = tok.apply_chat_template(msgs)
    assert ids == tok.encode(ct.render(msgs))


def test_template_helpers_behave_like_hf(tpl):
    src = "{{ messages | tojson }}{% generation %}[{{ messages[0].content }}]{% endgeneration %}"
    out = ct.render_jinja(src, [{"role": "user", "content": "ünï"}])
    assert out == '[{"role": "user", "content": "ünï"}][ünï]'
    with pytest.raises(Exception, match="boom"):
        ct.render_jinja("{{ raise_exception('boom') }}", [])
    assert ct.render_jinja("{{ bos_token }}|{{ eos_token }}", [], special_tokens={"bos_token": "<s>",
                                                                                 "eos_token": "</s>"}) == "<s>|</s>"


REF_PARQUET = "/root/reference/data/qa_dataset.parquet"


@pytest.mark.skipif(not os.path.exists(REF_PARQUET), reason="reference dataset not present")
def test_reference_rows_token_counts(tpl):
    """Token counts of the reference's own parquet rows through both template paths (synthetic BPE
    tokenizer: the real SmolLM3 vocabulary is not available offline, so absolute counts are unpinned)."""
    from llm_fine_tune_distributed_amd.data.dataset import load_qa_parquet
    rows = load_qa_parquet(REF_PARQUET)
    assert len(rows) == 2845
    tk = load_tokenizer(corpus=[r["full-question"] for r in rows] + [r["answer"] for r in rows])
    sample = rows[::57]
    n_builtin = [len(tk.apply_chat_template(format_prompt(r)["messages"])) for r in sample]
    tk.chat_template = tpl
    n_jinja = [len(tk.apply_chat_template(format_prompt(r)["messages"])) for r in sample]
    assert n_builtin == n_jinja
    assert 250 < min(n_builtin) and max(n_builtin) < 1024  # never truncated at max_seq_length=1024
