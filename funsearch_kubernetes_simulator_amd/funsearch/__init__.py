"""L4: FunSearch evolution -- LLM backends, reference-compatible loop, islands."""
from .funsearch_integration import evaluate_policy_standalone
from .generator import LLMCodeGenerator
from .islands import IslandFunSearch, run_funsearch
from .llm import MutationClient, OpenAICompatibleClient, ScriptedClient, make_client
from .scheduler import FunSearchScheduler
from .search import SimpleFunSearch

__all__ = ["evaluate_policy_standalone", "LLMCodeGenerator", "IslandFunSearch", "run_funsearch",
           "MutationClient", "OpenAICompatibleClient", "ScriptedClient", "make_client",
           "FunSearchScheduler", "SimpleFunSearch"]
