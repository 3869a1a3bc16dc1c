"""`LLMCodeGenerator`: prompt -> LLM -> template fill -> validation.

Same contract as the reference (`funsearch/safe_execution.py:273-317`): one
chat completion per call, the reply is the body that replaces
``{llm_generated_logic}``, the filled program must pass the content and
structure checks, and any failure yields ``None``.  Differences: the client
is any `llm.BaseClient` (HTTP with retries, offline mutation, scripted), a
markdown code fence around the reply is stripped instead of failing the
candidate, and per-call latency is recorded for the metrics log.
"""

from __future__ import annotations

import re
import time
from typing import List, Optional, Sequence, Tuple

from ..policy.sandbox import SafeExecutor
from ..policy.template import PolicyTemplate

_FENCE = re.compile(r"^```[a-zA-Z]*\n(.*?)\n?```\s*$", re.S)


class LLMCodeGenerator:
    def __init__(self, llm_client, safe_executor: Optional[SafeExecutor] = None, model: Optional[str] = None,
                 max_tokens: int = 400, temperature: float = 0.7, verbose: bool = False):
        self.llm_client = llm_client
        self.safe_executor = safe_executor or SafeExecutor()
        self.model = model or "gpt-3.5-turbo"
        self.max_tokens = max_tokens
        self.temperature = temperature
        self.verbose = verbose
        self.latencies: List[float] = []
        self.rejected = 0

    @staticmethod
    def clean_reply(text: str) -> str:
        text = text.strip()
        m = _FENCE.match(text)
        return m.group(1) if m else text

    def generate_policy(self, parent_policies: Optional[Sequence[Tuple[str, float]]] = None,
                        performance_feedback: str = "", prevalidated=None) -> Optional[str]:
        """prevalidated(code) -> True: the caller vouches for the code's safety
        (steady mode: a child that differs from an already-validated parent in
        numeric literal digits only), so the two checks are skipped."""
        prompt = PolicyTemplate.create_prompt_for_llm(parent_policies or [], performance_feedback)
        try:
            t0 = time.time()
            resp = self.llm_client.chat.completions.create(
                model=self.model, messages=[{"role": "user", "content": prompt}],
                temperature=self.temperature, max_tokens=self.max_tokens)
            self.latencies.append(time.time() - t0)
            logic = self.clean_reply(resp.choices[0].message.content)
            code = PolicyTemplate.fill_template(logic)
            if self.verbose:
                print(code)
            if prevalidated is None or not prevalidated(code):
                self.safe_executor.validate_code_content(code)
                self.safe_executor.validate_code_structure(code)
            return code
        except Exception as exc:
            self.rejected += 1
            if self.verbose:
                print(f"Error generating policy: {exc}")
            return None

    def test_policy_safely(self, code: str, test_pod, test_node) -> Optional[float]:
        try:
            return self.safe_executor.execute_policy_function(code, test_pod, test_node)
        except Exception as exc:
            if self.verbose:
                print(f"Error testing policy: {exc}")
            return None
