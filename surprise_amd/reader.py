"""Rating-file parsing, mirroring surprise/reader.py:9-104 and the reader
parameters of surprise/builtin_datasets.py:33-66 (download is out of scope:
there is no network; files are used only if already on disk)."""
import os
from collections import namedtuple
from os.path import join


def get_dataset_dir():
    """builtin_datasets.py:14-27: $SURPRISE_DATA_FOLDER or ~/.surprise_data/ (not created)."""
    return os.environ.get("SURPRISE_DATA_FOLDER", os.path.expanduser("~") + "/.surprise_data/")


BuiltinDataset = namedtuple("BuiltinDataset", ["url", "path", "reader_params"])

BUILTIN_DATASETS = {
    "ml-100k": BuiltinDataset(
        url="http://files.grouplens.org/datasets/movielens/ml-100k.zip",
        path=join(get_dataset_dir(), "ml-100k/ml-100k/u.data"),
        reader_params=dict(line_format="user item rating timestamp", rating_scale=(1, 5),
                           sep="\t")),
    "ml-1m": BuiltinDataset(
        url="http://files.grouplens.org/datasets/movielens/ml-1m.zip",
        path=join(get_dataset_dir(), "ml-1m/ml-1m/ratings.dat"),
        reader_params=dict(line_format="user item rating timestamp", rating_scale=(1, 5),
                           sep="::")),
    "ml-20m": BuiltinDataset(
        url="http://files.grouplens.org/datasets/movielens/ml-20m.zip",
        path=join(get_dataset_dir(), "ml-20m/ml-20m/ratings.csv"),
        reader_params=dict(line_format="user item rating timestamp", rating_scale=(0.5, 5.0),
                           sep=",")),
    "jester": BuiltinDataset(
        url="http://eigentaste.berkeley.edu/dataset/jester_dataset_2.zip",
        path=join(get_dataset_dir(), "jester/jester_ratings.dat"),
        reader_params=dict(line_format="user item rating", rating_scale=(-10, 10))),
}


class Reader:
    """Parse 'user item rating [timestamp]' lines (reader.py:9-104).

    Ratings are shifted by ``offset = 1 - lower_bound`` when the lower bound is
    <= 0 (reader.py:58-59), so that every stored rating is >= 1."""

    def __init__(self, name=None, line_format="user item rating", sep=None, rating_scale=(1, 5),
                 skip_lines=0):
        if name:
            try:
                self.__init__(**BUILTIN_DATASETS[name].reader_params)
            except KeyError:
                raise ValueError("unknown reader " + name + ". Accepted values are " +
                                 ", ".join(BUILTIN_DATASETS.keys()) + ".")
        else:
            self.sep = sep
            self.skip_lines = skip_lines
            self.rating_scale = rating_scale
            lower_bound, higher_bound = rating_scale
            self.offset = -lower_bound + 1 if lower_bound <= 0 else 0
            splitted_format = line_format.split()
            entities = ["user", "item", "rating"]
            if "timestamp" in splitted_format:
                self.with_timestamp = True
                entities.append("timestamp")
            else:
                self.with_timestamp = False
            if any(field not in entities for field in splitted_format):
                raise ValueError("line_format parameter is incorrect.")
            self.indexes = [splitted_format.index(entity) for entity in entities]

    def parse_line(self, line):
        """Return (uid, iid, rating + offset, timestamp) -- reader.py:77-104."""
        line = line.split(self.sep)
        try:
            if self.with_timestamp:
                uid, iid, r, timestamp = (line[i].strip() for i in self.indexes)
            else:
                uid, iid, r = (line[i].strip() for i in self.indexes)
                timestamp = None
        except IndexError:
            raise ValueError("Impossible to parse line. Check the line_format and sep parameters.")
        return uid, iid, float(r) + self.offset, timestamp
