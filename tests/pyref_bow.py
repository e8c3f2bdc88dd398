"""Independent pure-Python restatement of DBoW2 TemplatedVocabulary::transform(features, BowVector,
FeatureVector, levelsup) (ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1256) with dicts the way
the reference uses std::map.  Slow; small inputs.  Pins the C oracle (tests/test_oracle_dbow.py)."""
import math

import numpy as np


def forb_distance(a, b):
    return int(np.bitwise_count(np.bitwise_xor(a, b)).sum())


def children_of(voc):
    ch = {i: [] for i in range(voc.n_nodes)}
    for i in range(1, voc.n_nodes):
        ch[int(voc.parent[i])].append(i)  # loadFromTextFile: children.push_back in file order
    return ch


def word_ids(voc):
    w, out = 0, {}
    for i in range(1, voc.n_nodes):
        if voc.is_leaf[i]:
            out[i] = w
            w += 1
    return out


def transform_one(voc, ch, wid, f, levelsup):
    nid_level = voc.L - levelsup
    nid = 0
    final_id, level = 0, 0
    while True:
        level += 1
        nodes = ch[final_id]
        final_id = nodes[0]
        best_d = float(forb_distance(f, voc.desc[final_id]))
        for n in nodes[1:]:
            d = float(forb_distance(f, voc.desc[n]))
            if d < best_d:
                best_d, final_id = d, n
        if level == nid_level:
            nid = final_id
        if voc.is_leaf[final_id]:
            break
    return wid[final_id], float(voc.weight[final_id]), nid


def transform(voc, desc, levelsup=4):
    """Returns (bow: dict word -> value, fv: dict node -> [features])."""
    if voc.n_nodes <= 1:
        return {}, {}
    ch, wid = children_of(voc), word_ids(voc)
    bow, fv = {}, {}
    add = voc.weighting in (0, 1)  # TF_IDF, TF
    for i, f in enumerate(desc):
        w_id, w, nid = transform_one(voc, ch, wid, f, levelsup)
        if w > 0:
            if add:
                bow[w_id] = bow.get(w_id, 0.0) + w
            elif w_id not in bow:
                bow[w_id] = w
            fv.setdefault(nid, []).append(i)
    must = voc.scoring != 5
    l2 = voc.scoring == 1
    keys = sorted(bow)
    if add and bow and not must:
        nd = float(len(bow))
        for k in keys:
            bow[k] /= nd
    if must:
        if l2:
            norm = 0.0
            for k in keys:
                norm += bow[k] * bow[k]
            norm = math.sqrt(norm)
        else:
            norm = 0.0
            for k in keys:
                norm += abs(bow[k])
        if norm > 0:
            for k in keys:
                bow[k] /= norm
    return bow, fv
