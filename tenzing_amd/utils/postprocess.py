"""Design-rule mining from search results (reference postprocess/postprocess.py:25-771).

Pipeline, re-implemented on our result formats:

1. ``load_results``: results CSV (``i|p01|p10|p50|p90|p99|stddev|op-json|...``, optional leading
   JSON options line) or the JSONL written by ``SearchResult.dump_jsonl``.
2. ``performance_classes``: sort schedules by pct10, convolve with a +1/-1 step kernel and take
   the prominent peaks (scipy ``find_peaks``) as class boundaries — schedules between two jumps
   in run time form one performance class.
3. ``feature_matrix``: binary features per schedule — "A and B on the same stream" (GPU ops),
   "A before B" (graph ops), "op X present" (which ChoiceOp alternative was taken), plus stream
   count and sync-op count buckets.
4. ``train_rules``: an entropy decision tree (class-balanced), leaves grown while the training
   error keeps dropping; each root-to-leaf path is a human-readable rule for a class.
5. ``evaluate_rules``: train on the first n results (e.g. the first n MCTS iterations), test on
   all of them — how early the search reveals the rules.

``python -m tenzing_amd.utils.postprocess results.csv --out prefix_`` writes ``prefix_rules.txt``
and ``prefix_classes.json``; with ``--plots`` also the reference's figures (matplotlib):
``prefix_classes.pdf`` (sorted times, the step-kernel response and the class boundaries),
``prefix_tree.pdf`` (the decision tree) and ``prefix_eval.pdf`` (rule accuracy against the
number of results trained on).
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from dataclasses import dataclass, field

import numpy as np

SYNC_KINDS = {"CudaEventRecord", "CudaEventSync", "CudaStreamWaitEvent", "StreamSync", "StreamWait",
              "HipEventRecord", "HipEventSync", "HipStreamWaitEvent"}


@dataclass
class Result:
    i: int
    pct: dict
    seq: list = field(default_factory=list)

    @property
    def pct10(self) -> float:
        return self.pct["pct10"]


def _split_top(line: str, delim: str = "|"):
    out, cur, in_str, esc = [], [], False, False
    for c in line:
        if in_str:
            cur.append(c)
            if esc:
                esc = False
            elif c == "\\":
                esc = True
            elif c == '"':
                in_str = False
            continue
        if c == '"':
            in_str = True
        if c == delim:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(c)
    out.append("".join(cur))
    return out


def load_results(path: str) -> list[Result]:
    res = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith("{") and '"result"' in line:  # JSONL
                j = json.loads(line)
                res.append(Result(j["i"], j["result"], j["seq"]))
                continue
            if line.startswith("{") or line.startswith("#"):
                continue  # options header
            cols = _split_top(line)
            if len(cols) < 7:
                continue
            try:
                pct = dict(zip(["pct01", "pct10", "pct50", "pct90", "pct99", "stddev"],
                               map(float, cols[1:7])))
            except ValueError:
                continue
            res.append(Result(int(cols[0]), pct, [json.loads(c) for c in cols[7:]]))
    return res


def is_sync(op: dict) -> bool:
    return op.get("kind") in SYNC_KINDS


def performance_classes(times, radius_frac: float = 0.005, pctl: float = 99.0):
    """Class label per entry of ``times`` (in input order) from jumps in the sorted times."""
    from scipy.signal import find_peaks

    times = np.asarray(times, dtype=float)
    order = np.argsort(times, kind="stable")
    arr = times[order]
    n = len(arr)
    labels = np.zeros(n, dtype=int)
    if n < 4:
        return labels, []
    kr = max(1, int(math.ceil(n * radius_frac)))
    kernel = np.array([1.0] * kr + [-1.0] * kr)
    conv = np.convolve(arr, kernel, "valid")
    cutoff = np.percentile(conv, pctl)
    peaks, _ = find_peaks(conv, prominence=max(cutoff, 1e-15), width=1)
    bounds = sorted(int(p) + kr for p in peaks)
    cls_sorted = np.searchsorted(np.array(bounds), np.arange(n), side="right")
    labels[order] = cls_sorted
    return labels, bounds


def feature_matrix(results: list[Result]):
    gpu_ops, graph_ops, present = set(), set(), {}
    for r in results:
        for op in r.seq:
            if is_sync(op):
                continue
            graph_ops.add(op["name"])
            if "stream" in op:
                gpu_ops.add(op["name"])
            present[op["name"]] = present.get(op["name"], 0) + 1
    gpu_ops, graph_ops = sorted(gpu_ops), sorted(graph_ops)
    optional = sorted(k for k, v in present.items() if v < len(results))
    names = []
    cols = []
    # same stream (unordered pairs)
    pairs = [(a, b) for i, a in enumerate(gpu_ops) for b in gpu_ops[i + 1:]]
    # Start/Finish bracket every schedule: "Start before X" only restates "uses X"
    ends = ("Start", "Finish")
    order_pairs = [(a, b) for a in graph_ops for b in graph_ops
                   if a != b and a not in ends and b not in ends]
    # "uses X" first: of two identical columns the earlier name is kept, and the choice taken
    # is the most readable reason for a class
    for o in optional:
        names.append(f"uses {o}")
    for a, b in pairs:
        names.append(f"{a} and {b} same stream")
    for a, b in order_pairs:
        names.append(f"{a} before {b}")
    names += ["streams>=2", "streams>=3", "streams>=4"]
    X = np.zeros((len(results), len(names)), dtype=np.int8)
    for ri, r in enumerate(results):
        stream = {}
        pos = {}
        nsync = 0
        for k, op in enumerate(r.seq):
            if is_sync(op):
                nsync += 1
                continue
            if "stream" in op:
                stream[op["name"]] = op["stream"]
            pos.setdefault(op["name"], k)
        c = 0
        for o in optional:
            X[ri, c] = int(o in pos)
            c += 1
        for a, b in pairs:
            X[ri, c] = int(a in stream and b in stream and stream[a] == stream[b])
            c += 1
        for a, b in order_pairs:
            X[ri, c] = int(a in pos and b in pos and pos[a] < pos[b])
            c += 1
        ns = len(set(stream.values()))
        for t in (2, 3, 4):
            X[ri, c] = int(ns >= t)
            c += 1
    # drop constant and duplicate columns (reference remove_redundant_features)
    keep, seen = [], {}
    for j in range(X.shape[1]):
        col = X[:, j]
        if col.min() == col.max():
            continue
        key = col.tobytes()
        if key in seen:
            continue
        seen[key] = j
        keep.append(j)
    return X[:, keep], [names[j] for j in keep]


def train_rules(X, y, names, max_leaves: int = 64):
    from sklearn.tree import DecisionTreeClassifier

    best, best_err = None, math.inf
    for leaves in range(2, max_leaves + 1):
        clf = DecisionTreeClassifier(criterion="entropy", class_weight="balanced",
                                     max_leaf_nodes=leaves, random_state=0)
        clf.fit(X, y)
        err = float(np.mean(clf.predict(X) != y))
        if err < best_err - 1e-12:
            best, best_err = clf, err
        elif best is not None and leaves > 4:
            break
        if err == 0:
            break
    rules = extract_rules(best, names) if best is not None else []
    return best, best_err, rules


def extract_rules(clf, names):
    t = clf.tree_
    out = []

    def walk(node, conds):
        if t.children_left[node] == t.children_right[node]:  # leaf
            cls = int(clf.classes_[int(np.argmax(t.value[node]))])
            n = int(t.n_node_samples[node])
            out.append((cls, n, list(conds)))
            return
        f = names[t.feature[node]]
        walk(t.children_left[node], conds + [f"NOT ({f})"])
        walk(t.children_right[node], conds + [f"({f})"])

    walk(0, [])
    out.sort()
    return out


def evaluate_rules(results: list[Result], n: int, labels=None):
    """train on the first n results, accuracy on all"""
    if labels is None:
        labels, _ = performance_classes([r.pct10 for r in results])
    X, names = feature_matrix(results)
    if n >= len(results) or len(set(labels[:n])) < 2:
        return None
    from sklearn.tree import DecisionTreeClassifier

    clf = DecisionTreeClassifier(criterion="entropy", class_weight="balanced", random_state=0)
    clf.fit(X[:n], labels[:n])
    return float(np.mean(clf.predict(X) == labels))


def process(results: list[Result], pctl: float = 99.0, plots: str = ""):
    """classes, features, rules; ``plots``: file prefix for the figures ("" = none)"""
    labels, bounds = performance_classes([r.pct10 for r in results], pctl=pctl)
    X, names = feature_matrix(results)
    report = {"n": len(results), "classes": int(labels.max() + 1) if len(labels) else 0,
              "class_bounds_sorted_index": bounds}
    if plots and len(results):
        plot_classes([r.pct10 for r in results], labels, bounds, plots + "classes.pdf")
    if report["classes"] < 2 or X.shape[1] == 0:
        return report, []
    clf, err, rules = train_rules(X, labels, names)
    if plots and clf is not None:
        plot_tree(clf, names, plots + "tree.pdf")
    cls_times = {}
    for c in range(report["classes"]):
        ts = [r.pct10 for r, l in zip(results, labels) if l == c]
        cls_times[c] = (min(ts), max(ts), len(ts))
    report["train_error"] = err
    report["class_times"] = {str(k): v for k, v in cls_times.items()}
    return report, rules


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    from matplotlib import pyplot as plt

    return plt


def plot_classes(times, labels, bounds, path, radius_frac: float = 0.005):
    """Reference postprocess.py:25-101 figure: the sorted pct10 times coloured by class, the
    +1/-1 step-kernel response whose peaks are the class boundaries, and the boundaries."""
    plt = _plt()
    times = np.asarray(times, dtype=float) * 1e3
    order = np.argsort(times, kind="stable")
    arr = times[order]
    n = len(arr)
    kr = max(1, int(math.ceil(n * radius_frac)))
    conv = np.convolve(arr, np.array([1.0] * kr + [-1.0] * kr), "valid") if n > 2 * kr else np.zeros(0)
    fig, axs = plt.subplots(2, sharex=True, figsize=(5, 4))
    axs[0].scatter(np.arange(n), arr, c=np.asarray(labels)[order], s=4, cmap="tab10")
    axs[0].set_ylabel("pct10 (ms)")
    axs[1].plot(np.arange(len(conv)) + kr, conv, color="black", linewidth=0.8)
    axs[1].set_ylabel("step response")
    axs[1].set_xlabel("schedules, sorted by time")
    for b in bounds:
        for ax in axs:
            ax.axvline(b, color="gray", linestyle=":", linewidth=0.8)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def plot_tree(clf, names, path):
    """Reference postprocess.py:254-278 (predict_{depth}.pdf): the trained decision tree."""
    from sklearn.tree import plot_tree as sk_plot_tree

    plt = _plt()
    depth = clf.get_depth()
    fig, ax = plt.subplots(figsize=(max(6, 3 * clf.get_n_leaves()), max(4, 2 * depth)))
    sk_plot_tree(clf, feature_names=names, class_names=[str(c) for c in clf.classes_],
                 filled=True, impurity=False, ax=ax, fontsize=7)
    fig.savefig(path)
    plt.close(fig)


def plot_eval(evals: dict, path):
    """Reference postprocess.py:719-771 (eval_rules.pdf): accuracy on all results of the rules
    trained on the first n."""
    plt = _plt()
    pts = sorted((int(k), v) for k, v in evals.items() if v is not None)
    fig, ax = plt.subplots(figsize=(4, 2.5))
    if pts:
        ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", color="black")
    ax.set_xlabel("results trained on")
    ax.set_ylabel("accuracy on all")
    ax.set_ylim(0, 1.05)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def format_rules(rules, report) -> str:
    lines = []
    for cls, n, conds in rules:
        t = report.get("class_times", {}).get(str(cls))
        rng = f" [{t[0] * 1e3:.4f}-{t[1] * 1e3:.4f} ms]" if t else ""
        lines.append(f"class {cls}{rng} ({n} schedules): " + (" AND ".join(conds) or "always"))
    return "\n".join(lines) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("results")
    ap.add_argument("--out", default="")
    ap.add_argument("--pctl", type=float, default=99.0)
    ap.add_argument("--eval", type=int, nargs="*", default=[50, 100, 200, 400])
    ap.add_argument("--plots", action="store_true",
                    help="also write the figures (classes, tree, eval) as PDFs next to --out")
    a = ap.parse_args(argv)
    results = load_results(a.results)
    prefix = (a.out or "rules_") if a.plots else ""
    report, rules = process(results, a.pctl, plots=prefix)
    report["eval"] = {str(n): evaluate_rules(results, n) for n in a.eval if n < len(results)}
    if prefix:
        plot_eval(report["eval"], prefix + "eval.pdf")
    text = format_rules(rules, report)
    sys.stdout.write(text)
    if a.out:
        with open(a.out + "rules.txt", "w") as f:
            f.write(text)
        with open(a.out + "classes.json", "w") as f:
            json.dump(report, f, indent=1)
    print(json.dumps(report))
    return 0


if __name__ == "__main__":
    sys.exit(main())
