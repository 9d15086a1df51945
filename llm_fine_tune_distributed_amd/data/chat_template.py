"""Chat-template rendering (reference D3 / I1 / I2).

The reference delegates to ``tokenizer.apply_chat_template`` with the tokenizer's own template
(TRL, ``training.py:282-283``; ``ask_tuned_model.py:45-49``; ``enable_thinking=False`` at
``ask_original_model.py:44``). Two paths:

* ``render_jinja`` — when the tokenizer directory ships a template (``tokenizer_config.json``
  ``chat_template``, or a ``chat_template.jinja`` file) it is rendered with Jinja2 the way HF does:
  a sandboxed environment with ``trim_blocks`` / ``lstrip_blocks``, loop controls, a ``tojson``
  filter that keeps non-ASCII text, ``raise_exception`` / ``strftime_now`` globals, the special
  tokens as variables and every extra keyword (``enable_thinking``, ``xml_tools``...) passed
  through; ``{% generation %}`` blocks render their body.
* ``render`` — the built-in fallback for the offline synthetic tokenizer: ChatML in the SmolLM3
  style (system prompt in a metadata header, an empty think block for non-reasoning turns).
  Byte-parity of this fallback with the hub template is unpinned (the hub files are not available
  offline); ``tests/test_chat_template_cpu.py`` pins it against a fixture template of the same shape.
"""
from __future__ import annotations

from typing import Dict, List

IM_START, IM_END = "<|im_start|>", "<|im_end|>"
THINK_OPEN, THINK_CLOSE = "<think>", "</think>"


def render(messages: List[Dict[str, str]], add_generation_prompt: bool = False, enable_thinking: bool = False,
           metadata: bool = True, today: str = "01 January 2026") -> str:
    out = []
    sys_msgs = [m for m in messages if m["role"] == "system"]
    sys_text = sys_msgs[0]["content"] if sys_msgs else ""
    mode = "/think" if enable_thinking else "/no_think"
    if metadata:
        head = (f"## Metadata\n\nKnowledge Cutoff Date: June 2025\nToday Date: {today}\nReasoning Mode: {mode}\n\n"
                f"## Custom Instructions\n\n{sys_text}\n\n")
        out.append(f"{IM_START}system\n{head}{IM_END}\n")
    elif sys_text:
        out.append(f"{IM_START}system\n{sys_text}{IM_END}\n")
    for m in messages:
        if m["role"] == "system":
            continue
        if m["role"] == "assistant":
            body = m["content"]
            if not enable_thinking and THINK_OPEN not in body:
                body = f"{THINK_OPEN}\n\n{THINK_CLOSE}\n{body}"
            out.append(f"{IM_START}assistant\n{body}{IM_END}\n")
        else:
            out.append(f"{IM_START}{m['role']}\n{m['content']}{IM_END}\n")
    if add_generation_prompt:
        out.append(f"{IM_START}assistant\n")
        if not enable_thinking:
            out.append(f"{THINK_OPEN}\n\n{THINK_CLOSE}\n")
    return "".join(out)


def assistant_span(text: str) -> str:
    """Extract the assistant reply the way ask_tuned_model.py:67-90 does."""
    for marker in (f"{IM_START}assistant\n", f"{IM_START}assistant", "assistant\n", "assistant:", "<|assistant|>"):
        if marker in text:
            resp = text[text.rfind(marker) + len(marker):]
            if IM_END in resp:
                resp = resp.split(IM_END)[0]
            if THINK_CLOSE in resp:
                resp = resp.split(THINK_CLOSE, 1)[1]
            return resp.strip()
    return text.strip()


# ---------------------------------------------------------------------------- Jinja (tokenizer's own template)
_ENV_CACHE = {}


def _environment():
    if "env" in _ENV_CACHE:
        return _ENV_CACHE["env"]
    import json
    from datetime import datetime

    import jinja2
    from jinja2 import nodes
    from jinja2.ext import Extension
    from jinja2.sandbox import ImmutableSandboxedEnvironment

    class GenerationBlock(Extension):
        """``{% generation %}...{% endgeneration %}`` marks assistant text for HF's assistant masks; the
        body is rendered unchanged (masks come from ``assistant_only_loss`` instead)."""
        tags = {"generation"}

        def parse(self, parser):
            lineno = next(parser.stream).lineno
            body = parser.parse_statements(("name:endgeneration",), drop_needle=True)
            return nodes.Scope(body).set_lineno(lineno)

    def raise_exception(message):
        raise jinja2.exceptions.TemplateError(message)

    def tojson(x, ensure_ascii=False, indent=None, separators=None, sort_keys=False):
        return json.dumps(x, ensure_ascii=ensure_ascii, indent=indent, separators=separators, sort_keys=sort_keys)

    def strftime_now(fmt):
        return datetime.now().strftime(fmt)

    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True,
                                        extensions=[GenerationBlock, jinja2.ext.loopcontrols])
    env.filters["tojson"] = tojson
    env.globals["raise_exception"] = raise_exception
    env.globals["strftime_now"] = strftime_now
    _ENV_CACHE["env"] = env
    return env


def compile_template(source: str):
    key = ("tpl", source)
    if key not in _ENV_CACHE:
        _ENV_CACHE[key] = _environment().from_string(source)
    return _ENV_CACHE[key]


def render_jinja(source: str, messages: List[Dict[str, str]], add_generation_prompt: bool = False,
                 special_tokens: Dict[str, str] = None, **kwargs) -> str:
    """Render ``messages`` through a tokenizer's Jinja chat template (HF ``apply_chat_template`` semantics)."""
    variables = {k: v for k, v in (special_tokens or {}).items() if v is not None}
    variables.update(kwargs)
    variables.setdefault("tools", None)
    variables.setdefault("documents", None)
    return compile_template(source).render(messages=messages, add_generation_prompt=add_generation_prompt,
                                           **variables)


def select_template(cfg_template, name: str = "default"):
    """``tokenizer_config.json`` holds either one template string or a list of ``{name, template}``."""
    if cfg_template is None or isinstance(cfg_template, str):
        return cfg_template
    table = {t["name"]: t["template"] for t in cfg_template}
    return table.get(name) or table.get("default") or next(iter(table.values()), None)
