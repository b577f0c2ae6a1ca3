"""Chat templates of the local chat client (llama3 / mistral / chatml): turn layout, tool listing, the
score prompt's trailing system message, and the per-architecture default."""
import pytest

from llm_weighted_consensus_amd.chat.local import render_chat_prompt, template_for
from llm_weighted_consensus_amd.schema import chat as C

MSGS = [C.SystemMessage(content="be brief"), C.UserMessage(content="hi"), C.AssistantMessage(content="yo"),
        C.UserMessage(content="again"), C.SystemMessage(content="Select the response:\n\n{...}")]


def test_llama3_layout():
    p = render_chat_prompt(MSGS, None, "llama3")
    assert p.startswith("<|start_header_id|>system<|end_header_id|>\n\nbe brief<|eot_id|>")
    assert "<|begin_of_text|>" not in p  # BOS is an id added by the engine, not text
    assert p.endswith("Select the response:\n\n{...}<|eot_id|><|start_header_id|>assistant<|end_header_id|>\n\n")


def test_mistral_folds_turns_between_answers():
    p = render_chat_prompt(MSGS, None, "mistral")
    assert p == "[INST] be brief\n\nhi [/INST]yo</s>[INST] again\n\nSelect the response:\n\n{...} [/INST]"


def test_chatml_layout_and_tools():
    tool = C.Tool.model_validate({"type": "function", "function": {"name": "response_key", "parameters": {}}})
    p = render_chat_prompt(MSGS[:2], [tool], "chatml")
    assert p.startswith("<|im_start|>system\nAvailable tools: [")
    assert p.endswith("<|im_start|>user\nhi<|im_end|>\n<|im_start|>assistant\n")


def test_template_defaults_and_unknown():
    assert template_for("llama-3-8b") == "llama3"
    assert template_for("mixtral-8x7b") == "mistral" and template_for("e5-mistral-7b") == "mistral"
    with pytest.raises(ValueError):
        render_chat_prompt(MSGS, None, "nope")
