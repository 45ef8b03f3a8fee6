"""Pickle (predictions, algo), mirroring surprise/dump.py:8-58.  Fitted SVD/SVDpp
objects pickle their factors as host numpy arrays (no device handles)."""
import pickle


def dump(file_name, predictions=None, algo=None, verbose=0):
    dump_obj = {"predictions": predictions, "algo": algo}
    with open(file_name, "wb") as f:
        pickle.dump(dump_obj, f, protocol=pickle.HIGHEST_PROTOCOL)
    if verbose:
        print("The dump has been saved as file", file_name)


def load(file_name):
    # loads only files written by dump() above (this package's own objects)
    with open(file_name, "rb") as f:
        dump_obj = pickle.load(f)
    return dump_obj["predictions"], dump_obj["algo"]
