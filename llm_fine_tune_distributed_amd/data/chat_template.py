"""ChatML rendering in the SmolLM3 style (``<|im_start|>role\\n...<|im_end|>``).

The reference delegates to ``tokenizer.apply_chat_template`` with the hub template
(TRL, training.py:282-283; ask_tuned_model.py:44-48). SmolLM3's template wraps the system
prompt in a metadata header and emits an empty think block for non-reasoning turns; we
render the same structure without Jinja. Exact byte-parity with the hub template is
unpinned (the template file is not available offline); token counts match within the
header's few tokens.
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
