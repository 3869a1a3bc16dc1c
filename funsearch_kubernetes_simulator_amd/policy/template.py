"""Prompt / program template shared with LLM backends.

The template body and prompt wording are kept *verbatim* from the reference
(`funsearch/safe_execution.py:171-270`): they are part of the program-text
compatibility contract (the feasibility prologue is what every evolved policy
starts with, and prompts built here must read exactly like the ones that
produced the published champions).
"""

from __future__ import annotations

from typing import Iterable, Sequence, Tuple

_DOC = '''    """
    Calculate priority score for placing pod on node.
    Higher score = better placement.
    
    ## Data Structure Definitions

    # Pod Object
    # A 'pod' represents a workload request with specific resource requirements.
    - pod.cpu_milli (int): CPU requested in thousandths of a core.
    - pod.memory_mib (int): Memory requested in Mebibytes.
    - pod.num_gpu (int): The number of individual GPUs required.
    - pod.gpu_milli (int): The compute power required from each GPU.

    # Node Object
    # A 'node' represents a single machine in the cluster that can host pods.
    - node.cpu_milli_left (int): Remaining available CPU on the node.
    - node.memory_mib_left (int): Remaining available memory on the node.
    - node.gpu_left (int): The count of available (unassigned) GPUs.
    - node.cpu_milli_total (int): Total CPU capacity of the node.
    - node.memory_mib_total (int): Total memory capacity of the node.
    - node.gpus (list[GPU]): A list of 'GPU' objects available on this node.

    # GPU Object
    # A 'gpu' object represents a single GPU. These are found inside the 'node.gpus' list.
    - gpu.gpu_milli_left (int): Remaining available compute on this specific GPU.
    - gpu.gpu_milli_total (int): Total compute capacity of this GPU.
    """'''

#: Feasibility prologue every template-filled program starts with.
FEASIBILITY_PROLOGUE = '''    # Basic feasibility check
    if (pod.cpu_milli > node.cpu_milli_left or 
        pod.memory_mib > node.memory_mib_left or 
        pod.num_gpu > node.gpu_left):
        return 0
    
    if pod.num_gpu > 0:
        available_gpus = 0
        for gpu in node.gpus:
            if gpu.gpu_milli_left >= pod.gpu_milli:
                available_gpus += 1
        if available_gpus < pod.num_gpu:
            return 0'''


class PolicyTemplate:
    TEMPLATE = ("\ndef priority_function(pod, node):\n" + _DOC + "\n    \n" + FEASIBILITY_PROLOGUE
                + "\n    \n    # LLM fills in this part\n    score = 0.0\n    \n"
                + "    {llm_generated_logic}\n    \n    return max(1, int(score))\n")

    @classmethod
    def _format_parent_policies(cls, policies: Sequence[Tuple[str, float]]) -> str:
        if not policies:
            return "No previous policies available."
        return "".join(f"\nPolicy v_{i + 1} (score: {score:.3f}):\n{code}\n"
                       for i, (code, score) in enumerate(policies))

    @classmethod
    def create_prompt_for_llm(cls, parent_policies: Iterable[Tuple[str, float]],
                              performance_feedback: str) -> str:
        parents = cls._format_parent_policies(list(parent_policies))
        return (
            "\nYou are generating a kubernetes scheduling policy function. You must ONLY fill in the "
            "logic between the comments.\n\nCONSTRAINTS:\n"
            "- Only use basic math operations (+, -, *, /, %, **, abs, min, max)\n"
            "- Only use the provided variables: pod, node, cluster_state\n"
            "- No imports, no function definitions, no loops\n"
            "- Return a single numeric score\n"
            "- Use if/else statements if needed\n"
            "- Your generation should have nothing other than the code itself, do not output anything "
            "else. (Do not wrap in ```python)\n"
            "- IMPORTANT: Every line of code MUST start with exactly 4 spaces for proper indentation\n"
            "- Lines inside if/else blocks should start with 8 spaces, nested blocks with 12 spaces, etc.\n"
            f"\nTemplate to complete:\n{cls.TEMPLATE}\n"
            f"\nPrevious policies and their performance:\n{parents}\n"
            f"\nPerformance feedback: {performance_feedback}\n"
            "\nGenerate ONLY the logic to replace {llm_generated_logic}, nothing else.\n"
            "Remember: Each line must start with proper indentation (4 spaces minimum):\n"
        )

    @classmethod
    def fill_template(cls, llm_generated_logic: str) -> str:
        return cls.TEMPLATE.format(llm_generated_logic=llm_generated_logic.strip())

    @classmethod
    def extract_logic(cls, program: str) -> str:
        """Inverse of `fill_template` for template-shaped programs: the body
        between ``score = 0.0`` and the final ``return`` (used by mutation
        backends and prompt building)."""
        head = "    score = 0.0\n    \n"
        tail = "\n    \n    return max(1, int(score))\n"
        i, j = program.find(head), program.rfind(tail)
        if i < 0 or j < 0 or j < i:
            raise ValueError("program is not template-shaped")
        return program[i + len(head):j]
