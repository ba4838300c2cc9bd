"""Model IO and logging helpers the pruning path calls (counterpart of ResNet/utils.py).

The CSV schemas, header strings, directory convention and printed messages are outputs of
the reference path (utils.py:41-162), so they are reproduced exactly; nothing here is
accelerated.  load_model/save_model use Hugging Face transformers when the model is a
PreTrainedModel; plain nn.Modules are saved as a safetensors state_dict instead.
"""
import csv
import os

LAYER_LOG_FIELDS = ["GUID", "Wavelet", "Level", "Threshold", "DWT Phase", "Original Parameter Count",
                    "Non-zero Params", "Total Pruned Count", "Layer Name"]          # utils.py:55-58
EXPERIMENT_LOG_FIELDS = ["GUID", "Wavelet", "Level", "Threshold", "Phase", "Total Pruned Count",
                         "Total Non-Zero Params", "Model Path"]                      # utils.py:127-128


def load_model(model_path, config_path):
    """Load a local Hugging Face image-classification checkpoint (utils.py:6-25)."""
    if not os.path.isdir(model_path):
        raise ValueError(f"Provided model path {model_path} is not a valid directory.")
    from transformers import AutoConfig, AutoModelForImageClassification
    cfg = AutoConfig.from_pretrained(config_path)
    model = AutoModelForImageClassification.from_pretrained(model_path, config=cfg)
    print("Pre-trained model loaded successfully.")
    return model


def save_model(model, output_path):
    """save_pretrained into cwd/output_path (utils.py:28-38)."""
    target = os.path.normpath(os.path.join(os.getcwd(), output_path))
    if hasattr(model, "save_pretrained"):
        model.save_pretrained(target)
    else:
        from safetensors.torch import save_file
        os.makedirs(target, exist_ok=True)
        save_file({k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()},
                  os.path.join(target, "model.safetensors"))
    print(f"Model saved successfully at {target}")


def setup_csv_writer(file_path, mode="w"):
    """Open a per-layer log; header when writing fresh or appending to a new file (utils.py:41-65)."""
    try:
        existed = os.path.isfile(file_path)
        fh = open(file_path, mode=mode, newline="")
        writer = csv.DictWriter(fh, fieldnames=LAYER_LOG_FIELDS)
        if mode == "w" or (mode == "a" and not existed):
            writer.writeheader()
        return writer, fh
    except Exception as exc:
        print(f"Failed to set up CSV writer: {exc}")
        raise


def log_pruning_details(csv_writer, guid, wavelet, level, threshold, phase, original_param_count,
                        non_zero_params, total_pruned_count, layer_name):
    """One row of the per-layer log (utils.py:68-101)."""
    if not csv_writer or not layer_name:
        return
    values = [guid, wavelet, level, threshold, phase, original_param_count, non_zero_params,
              total_pruned_count, layer_name]
    try:
        csv_writer.writerow(dict(zip(LAYER_LOG_FIELDS, values)))
    except Exception as exc:
        print(f"Failed to log pruning details for layer {layer_name}: {exc}")


def append_to_experiment_log(file_path, guid, wavelet, level, threshold, phase, total_pruned_count,
                             total_non_zero_params, model_path):
    """Append one run summary to the experiment log, header on first write (utils.py:104-145)."""
    if not file_path:
        print("Error: Invalid file path provided.")
        return
    try:
        path = os.path.normpath(file_path)
        fresh = not os.path.isfile(path)
        with open(path, mode="a", newline="") as fh:
            writer = csv.DictWriter(fh, fieldnames=EXPERIMENT_LOG_FIELDS)
            if fresh:
                writer.writeheader()
            writer.writerow(dict(zip(EXPERIMENT_LOG_FIELDS, [guid, wavelet, level, threshold, phase,
                                                             total_pruned_count, total_non_zero_params,
                                                             model_path])))
    except Exception as exc:
        print(f"Error: Failed to append to experiment log: {exc}")


def check_and_set_pruned_instance_path(pruned_instance):
    """<cwd>/../../WaveletTransforms/ResNet/SavedModels/<pruned_instance>, created (utils.py:148-162)."""
    root = os.path.abspath(os.path.join(os.getcwd(), "../.."))
    path = os.path.join(root, "WaveletTransforms", "ResNet", "SavedModels", pruned_instance)
    print(f"Pruned instance path: {path}")
    os.makedirs(path, exist_ok=True)
    return path


def print_model_summary(model):
    """Top-level layers with a weight, their shapes and parameter counts (utils.py:165-188)."""
    total = 0
    print("Model Summary:")
    print("Layer Name" + "\t" * 7 + "Output Shape" + "\t" * 5 + "Param #")
    print("=" * 100)
    for name, child in model.named_children():
        w = getattr(child, "weight", None)
        if w is None or not hasattr(w, "size"):
            continue
        total += w.numel()
        b = getattr(child, "bias", None)
        if b is not None and hasattr(b, "size"):
            total += b.numel()
        print(f"{name}\t{w.size()}\t{w.numel()}")
    print("=" * 100)
    print(f"Total Params: {total}")


def print_model_structure(model, depth=0):
    """Indented module tree (utils.py:191-206)."""
    pad = "  " * depth
    for name, child in model.named_children():
        print(f"{pad}{name} - {child.__class__.__name__}")
        if any(True for _ in child.children()):
            print_model_structure(child, depth + 1)


def get_layer(model, layer_name):
    """Resolve a dotted layer name, tolerating a 'ResNetForImageClassification.' prefix (utils.py:209-237)."""
    prefix = "ResNetForImageClassification."
    if layer_name.startswith(prefix):
        layer_name = layer_name[len(prefix):]
    node = model
    for depth, part in enumerate(layer_name.split(".")):
        if not part:
            continue
        print(f"Checking for part '{part}' at level {depth}")
        if not hasattr(node, part):
            print(f"Layer part '{part}' not found in the model at level {depth}")
            return None
        node = getattr(node, part)
        print(f"Found part '{part}', current model: {type(node)}")
    return node
