"""Host logic of the layer-by-layer calibration flow (calibration.capture_layer_inputs /
propagate_layer, PT2LLMQuantizer.quantize(propagate="layerwise")) on CPU: the inputs each decoder
layer receives through layer-wise propagation are the hidden states the reference's full-model
forward hands it (main.py:280-282), so the flow quantises the same activations.  No kernels run
here; the GPU equivalence of the whole flow is test_gpu_model.py's."""
import pytest
import torch


def tiny_llama(layers=3):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(hidden_size=64, intermediate_size=96, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=4, vocab_size=101, max_position_embeddings=64)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval()


def full_forward_inputs(model, layer, samples):
    """The hidden state `layer` receives in a full forward of each sample (pre-hook capture)."""
    got = []

    def hook(mod, args, kwargs):
        got.append((args[0] if args else kwargs["hidden_states"]).clone())

    h = layer.register_forward_pre_hook(hook, with_kwargs=True)
    with torch.no_grad():
        for s in samples:
            model(s, use_cache=False)
    h.remove()
    return got


@pytest.mark.parametrize("perturb", [False, True])
def test_layerwise_propagation_matches_full_forward(pt2q, perturb):
    """Layer l's recorded inputs after propagating layers < l equal the full forward's, also after
    the earlier layers' weights were rewritten (the quantised write-back happens between layers)."""
    model = tiny_llama(3)
    layers = model.model.layers
    g = torch.Generator().manual_seed(1)
    samples = [torch.randint(0, 101, (1, 16), generator=g) for _ in range(3)]
    cal = pt2q.calibration
    with torch.no_grad():
        inputs = cal.capture_layer_inputs(model, layers[0], samples)
        assert len(inputs) == 3
        for l in range(len(layers)):
            want = full_forward_inputs(model, layers[l], samples)
            for (args, kwargs), w in zip(inputs, want):
                x = args[0] if args else kwargs["hidden_states"]
                assert torch.equal(x, w)
            if perturb:  # a stand-in for the write-back of layer l
                for lin in cal.find_linear_layers(layers[l]).values():
                    lin.weight.mul_(0.5)
            inputs = cal.propagate_layer(layers[l], inputs)


def test_capture_stops_at_the_layer(pt2q):
    """Only the layers before the recorded one run (the catcher stops the forward)."""
    model = tiny_llama(2)
    ran = []
    hs = [lay.register_forward_hook(lambda m, i, o, k=k: ran.append(k)) for k, lay in enumerate(model.model.layers)]
    pt2q.calibration.capture_layer_inputs(model, model.model.layers[1], [torch.zeros((1, 8), dtype=torch.long)])
    for h in hs:
        h.remove()
    assert ran == [0]
