"""pt2q — MI355X-native ternary PTQ calibration engine (PT²-LLM: ATQ + SSR inside a GPTQ loop).

Drop-in for the reference's hot-path surface:
    AsymmetricTernaryQuantizer, compute_quantization_error, compute_output_error  (quantizer.py)
    compute_column_similarity_to_mean, select_next_block_ssr                      (reorder.py)
    GPTQ, GPTQQuantizer                                                            (gptq.py)
    PT2LLMQuantizer.quantize_layer                                                 (main.py)
    pack_ternary, unpack_ternary, save/load_quantized_model,
    compute_bits_per_weight, evaluate_perplexity                                   (utils.py)
    TernaryLinear, replace_linear_with_ternary                                     (model.py)
All compute runs in libpt2q.so (HIP, gfx950); importing fails loudly if it is not built.
"""
from . import _lib
from .quantizer import AsymmetricTernaryQuantizer, compute_output_error, compute_quantization_error
from .reorder import compute_column_similarity_to_mean, select_next_block_ssr
from .gptq import GPTQ, GPTQQuantizer
from .pt2llm import PT2LLMQuantizer
from .calibration import (GramAccumulator, GramCapture, find_linear_layers, get_llm_layers,
                          quantize_decoder_layer)
from .ternary import (TernaryLinear, compute_bits_per_weight, load_quantized_model,
                      replace_linear_with_ternary, save_quantized_model)
from .evaluation import evaluate_perplexity
from .engine import (LayerGraph, LayerOutput, LayerWorkspace, UnitRun, UnitWorkspace, cholesky_inverse,
                     dequantize, error_feedback, fill_synthetic, gram, hessian_inverse, pack_ternary, prepare_hessian,
                     quantize_blocks, quantize_layer, quantize_shared, quantize_unit, unpack_ternary,
                     UnitPipeline, sum_partials)

__version__ = "0.1.0"
__all__ = [
    "AsymmetricTernaryQuantizer", "compute_quantization_error", "compute_output_error",
    "compute_column_similarity_to_mean", "select_next_block_ssr", "GPTQ", "GPTQQuantizer",
    "PT2LLMQuantizer", "LayerGraph", "LayerOutput", "LayerWorkspace", "gram", "prepare_hessian",
    "cholesky_inverse", "quantize_blocks", "quantize_layer", "dequantize", "pack_ternary",
    "unpack_ternary", "fill_synthetic", "hessian_inverse", "quantize_shared", "GramAccumulator",
    "GramCapture", "find_linear_layers", "get_llm_layers", "quantize_decoder_layer",
    "TernaryLinear", "replace_linear_with_ternary", "save_quantized_model", "load_quantized_model",
    "UnitRun", "UnitWorkspace", "quantize_unit", "compute_bits_per_weight", "error_feedback",
    "UnitPipeline", "sum_partials", "evaluate_perplexity",
]
