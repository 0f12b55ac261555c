"""Ablation studies (maggy.ablation.AblationStudy + the LOCO ablator).

Reference usage: notebooks/ml/Parallel_Experiments/Maggy/maggy-ablation-titanic-example.ipynb
(AblationStudy(name, training_dataset_version=1, label_name=…) :135, features.include :160-170,
model.set_base_model_generator :214, layers.include / include_groups(prefix=…) :240-300,
add_custom_model_generator :330, lagom(experiment_type='ablation', ablator='loco') :455).

LOCO = leave one component out: one trial with everything (``base``), then one
trial per included feature / layer / layer group with that component removed,
plus one trial per custom model.  Every trial is an independent process pinned
to one GPU (the trials of a study run concurrently, one per MI355X).

The training function receives ``dataset_function(epochs, batch_size)`` — an
iterable of (features, label) batches read from the feature store training
dataset (columns minus the label and the ablated feature) — and
``model_function()`` — the base model (a lazy :class:`hops_examples_amd.keras.Sequential`)
with the ablated layers removed, so the remaining layers re-infer their input sizes.
"""
from __future__ import annotations

import numpy as np


class _Features:
    def __init__(self):
        self.included: list[str] = []

    def include(self, *names):
        for n in names:
            for x in ([n] if isinstance(n, str) else list(n)):
                if x not in self.included:
                    self.included.append(x)

    def exclude(self, *names):
        for n in names:
            for x in ([n] if isinstance(n, str) else list(n)):
                if x in self.included:
                    self.included.remove(x)

    def list_all(self):
        for f in self.included:
            print(f)


class _Layers:
    def __init__(self):
        self.included: list[str] = []
        self.groups: list[tuple[str, tuple]] = []  # (label, ('list', names) | ('prefix', p))

    def include(self, *names):
        for n in names:
            for x in ([n] if isinstance(n, str) else list(n)):
                if x not in self.included:
                    self.included.append(x)

    def exclude(self, *names):
        for n in names:
            if n in self.included:
                self.included.remove(n)

    def include_groups(self, *groups, prefix: str | None = None):
        if prefix is not None:
            self.groups.append((f"prefix {prefix}", ("prefix", prefix)))
        for g in groups:
            g = list(g)
            if len(g) < 2:
                raise ValueError("a layer group needs at least two layers (use include() for one)")
            self.groups.append((f"group {g}", ("list", tuple(g))))

    def print_all(self):
        print("Included single layers are: \n")
        for n in self.included:
            print(n)

    def print_all_groups(self):
        print("Included layer groups are: \n")
        for label, _ in self.groups:
            print(label)


class _Model:
    def __init__(self):
        self.layers = _Layers()
        self.base_model_generator = None
        self.custom_model_generators: list[tuple] = []

    def set_base_model_generator(self, fn):
        self.base_model_generator = fn

    def add_custom_model_generator(self, fn, name: str):
        self.custom_model_generators.append((fn, name))


class AblationStudy:
    def __init__(self, training_dataset_name: str, training_dataset_version: int = 1, label_name: str | None = None,
                 **kwargs):
        self.hops_training_dataset_name = training_dataset_name
        self.hops_training_dataset_version = training_dataset_version
        self.label_name = label_name
        self.features = _Features()
        self.model = _Model()
        self.custom_dataset_generator = kwargs.get("dataset_generator")

    def set_dataset_generator(self, fn):
        """Override the feature-store reader: ``fn(ablated_feature, epochs, batch_size)`` -> batches."""
        self.custom_dataset_generator = fn

    def to_dict(self):
        return {"training_dataset": self.hops_training_dataset_name, "version": self.hops_training_dataset_version,
                "label": self.label_name, "features": list(self.features.included),
                "layers": list(self.model.layers.included), "groups": [g for g, _ in self.model.layers.groups],
                "custom_models": [n for _, n in self.model.custom_model_generators]}


# ---------------------------------------------------------------------------- trial factories


def _dataset_fn(study_dict: dict, ablated_feature: str | None, custom=None):
    name, version, label = study_dict["training_dataset"], study_dict["version"], study_dict["label"]

    def dataset_function(epochs: int = 1, batch_size: int = 32, shuffle: bool = True, seed: int = 0):
        if custom is not None:
            return custom(ablated_feature, epochs, batch_size)
        from ..featurestore import store as S

        fs = S.connection_quiet().get_feature_store()
        df = fs.get_training_dataset(name, version).read()
        cols = [c for c in df.columns if c != label and c != ablated_feature]
        x = df[cols].to_numpy(dtype=np.float32)
        y = df[label].to_numpy(dtype=np.float32)
        rng = np.random.default_rng(seed)

        def gen():
            for _ in range(epochs):
                idx = rng.permutation(len(x)) if shuffle else np.arange(len(x))
                for s in range(0, len(idx) - batch_size + 1, batch_size):
                    j = idx[s:s + batch_size]
                    yield x[j], y[j]

        return gen()

    return dataset_function


def _model_fn(generator, drop: tuple):
    def model_function():
        m = generator()
        if not drop:
            return m
        specs = getattr(m, "_specs", None)
        if specs is None:
            raise TypeError("layer ablation needs a hops_examples_amd.keras.Sequential base model")
        kept = []
        for l in specs:
            name = l.name
            gone = any((kind == "name" and name == v) or (kind == "prefix" and name.startswith(v)) or
                       (kind == "list" and name in v) for kind, v in drop)
            if not gone:
                kept.append(l)
        m._specs = kept
        return m

    return model_function


def trial_generators(study: AblationStudy, ablator: str = "loco"):
    """[(trial_name, {'dataset_function': f, 'model_function': g})] for the LOCO ablator."""
    if ablator.lower() != "loco":
        raise ValueError(f"unsupported ablator {ablator!r} (loco)")
    if study.model.base_model_generator is None:
        raise ValueError("set_base_model_generator() first")
    sd = study.to_dict()
    custom = study.custom_dataset_generator
    base = study.model.base_model_generator
    trials = [("base", {"dataset_function": _dataset_fn(sd, None, custom), "model_function": _model_fn(base, ())})]
    for f in study.features.included:
        trials.append((f"feature-{f}", {"dataset_function": _dataset_fn(sd, f, custom),
                                        "model_function": _model_fn(base, ())}))
    for l in study.model.layers.included:
        trials.append((f"layer-{l}", {"dataset_function": _dataset_fn(sd, None, custom),
                                      "model_function": _model_fn(base, (("name", l),))}))
    for label, (kind, v) in study.model.layers.groups:
        tname = "layers-" + (f"prefix-{v}" if kind == "prefix" else "-".join(v))
        trials.append((tname, {"dataset_function": _dataset_fn(sd, None, custom),
                               "model_function": _model_fn(base, ((kind, v),))}))
    for gen, name in study.model.custom_model_generators:
        trials.append((f"model-{name.replace(' ', '_')}", {"dataset_function": _dataset_fn(sd, None, custom),
                                                           "model_function": _model_fn(gen, ())}))
    return trials
