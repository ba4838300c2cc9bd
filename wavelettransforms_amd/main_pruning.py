"""The caller of the path, as ResNet/main_pruning.py (iAmGiG/WaveletTransforms) runs it, over this
package: load -> DWT (selective) pruning on the GPU -> the random and min-weight baselines in two
host threads that share one logging queue drained by a worker thread (main_pruning.py:104-215).

The flags mirror the reference's absl flags (main_pruning.py:83-102; absl is not part of this
image, so argparse reads the same names), with the wavelet list widened to every name the library
accepts (bior3.3 and db8 are BASELINE configs but absent from the reference's enum).  The
orchestration is `run()`, usable on an in-memory model.
"""
import argparse
import copy
import os
import queue
import threading

from .dwt_pruning import wavelet_pruning
from .min_weight_pruning import min_weight_pruning
from .random_pruning import random_pruning
from .utils import append_to_experiment_log, load_model

__all__ = ["log_worker", "threaded_pruning", "run", "main"]


def log_worker(csv_path, log_queue):
    """Append every queued run summary to the experiment log until a None arrives
    (main_pruning.py:108-115)."""
    while True:
        entry = log_queue.get()
        if entry is None:
            break
        append_to_experiment_log(csv_path, *entry)
        log_queue.task_done()


def threaded_pruning(pruning_func, model, selective_log_path, guid, wavelet, level, threshold, csv_path,
                     method_name, log_queue):
    """Run one baseline, report completion, swallow and print its error (main_pruning.py:118-127)."""
    try:
        result = pruning_func(model, selective_log_path, guid, wavelet, level, threshold, csv_path, log_queue)
        print(f"{method_name} pruning completed.")
        return result
    except Exception as e:  # the reference's contract: a failed baseline does not stop the run
        print(f"Error in {method_name} pruning: {str(e)}")
        return None


def run(model, wavelet, level, threshold, csv_path, guid=None):
    """main_pruning.py:169-215 on a loaded model: three deep copies, the selective (DWT) prune on
    the main thread, then random and min-weight pruning in two threads logging through one queue.
    Returns (guid, selective log path, (dwt, random, min) models)."""
    if guid is None:
        print("Generating Guid")
        guid = os.urandom(4).hex()
        print(f"Generated GUID: {guid}")
    print("Storing Deep copy of model")
    dwt_model = copy.deepcopy(model)
    random_model = copy.deepcopy(model)
    min_weight_model = copy.deepcopy(model)

    log_queue = queue.Queue()
    log_thread = threading.Thread(target=log_worker, args=(csv_path, log_queue))
    log_thread.start()
    try:
        print("Starting Selective (DWT) Pruning")
        selective_log_path = wavelet_pruning(dwt_model, wavelet, level, threshold * 100, csv_path, guid)
        print(f"Selective pruning completed. Log saved at {selective_log_path}")

        print("Starting Random pruning")
        random_thread = threading.Thread(
            target=threaded_pruning,
            args=(random_pruning, random_model, selective_log_path, guid, wavelet, level, threshold, csv_path,
                  "Random", log_queue))
        print("Starting Min weight pruning")
        min_weight_thread = threading.Thread(
            target=threaded_pruning,
            args=(min_weight_pruning, min_weight_model, selective_log_path, guid, wavelet, level, threshold,
                  csv_path, "Minimum Weight", log_queue))
        random_thread.start()
        min_weight_thread.start()
        random_thread.join()
        min_weight_thread.join()
    finally:
        log_queue.put(None)
        log_thread.join()
    print("All pruning methods completed successfully.")
    return guid, selective_log_path, (dwt_model, random_model, min_weight_model)


def main(argv=None):
    ap = argparse.ArgumentParser(description="DWT / random / min-weight pruning of a Hugging Face ResNet")
    ap.add_argument("--model_path", default="__OGPyTorchModel__/OGModel")
    ap.add_argument("--config_path", default="__OGPyTorchModel__/OGModel")
    ap.add_argument("--csv_path", default="experiment_log.csv")
    ap.add_argument("--wavelet", default="bior4.4")
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--threshold", type=float, default=0.1)
    ap.add_argument("--output_dir", default="SavedModels")  # unused, as in the reference
    a = ap.parse_args(argv)
    print(f"Model directory: {a.model_path}")
    print(f"Config file: {a.config_path}")
    if not os.path.isdir(a.model_path):
        raise ValueError(f"Provided model path {a.model_path} is not a valid directory.")
    model = load_model(a.model_path, a.config_path)
    print("Model loaded successfully.")
    run(model, a.wavelet, a.level, a.threshold, a.csv_path)


if __name__ == "__main__":
    main()
