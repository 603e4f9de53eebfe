"""ORACLE (test infrastructure only): literal restatement of GreedyStrategy's compute_fn.

Follows tneq_qc/contractor/greedy_strategy.py:41-1080 step by step, with numpy.einsum standing
in for torch.einsum (same equation strings after the reference's symbol remap):
  Step 1   core_tensor_list of L cores / L states / Mx / R cores / R states   :73-295
  Step 2   neighbour wiring                                                    :301-406
  Step 2.5 symbol assignment skipping 'a','b'                                  :411-449
  Step 3   per-qubit groups (scan + circuit-state pull-in + union-find)        :461-585
           _contract_symmetric_group incl. the R-side dim map                  :690-990
  Step 4   _contract_remaining                                                 :993-1080
Plain arrays only (TNTensor scale products are checked separately).  Returns the raw result
(before EngineSiamese's abs_square).
"""
from __future__ import annotations

from copy import deepcopy
from typing import Dict, List

import numpy as np

from .qctn_ref import QCTNRef, get_symbol

LEFT, MIDDLE, RIGHT = "L", "M", "R"


def _get_tensor(entry, cores, states, mx):                            # :667-687
    if "tensor" in entry:
        return entry["tensor"]
    src, key = entry["tensor_source"], entry["tensor_key"]
    if src == "core":
        return cores[key]
    if src == "transpose":
        return cores[key].conj() if np.iscomplexobj(cores[key]) else cores[key]
    if src == "circuit":
        return states[key]
    if src == "mx":
        return mx[key]
    raise ValueError(f"Unknown tensor source: {src}")


def _has(container, q):
    if container is None:
        return False
    if isinstance(container, dict):
        return q in container
    return q < len(container)


def greedy_contract(qctn: QCTNRef, cores: Dict[str, np.ndarray], states, mx, right_qctn="symmetric",
                    right_cores=None):
    cores = dict(cores)
    L: List[dict] = []

    # ---- Step 1
    left_core_map = {}
    for info in qctn.adjacency_table:
        uid = len(L)
        left_core_map[info["core_idx"]] = uid
        L.append({"core_idx": uid, "core_name": f"{info['core_name']}_L", "tensor_source": "core",
                  "tensor_key": info["core_name"], "in_edge_list": deepcopy(info["in_edge_list"]),
                  "out_edge_list": deepcopy(info["out_edge_list"]), "side": LEFT, "batch_symbol": ""})
    left_circuit_map = {}
    for q in qctn.qubit_indices:
        if not _has(states, q):
            continue
        uid = len(L)
        left_circuit_map[q] = uid
        L.append({"core_idx": uid, "core_name": f"circuit_L_{q}", "tensor_source": "circuit", "tensor_key": q,
                  "in_edge_list": [], "out_edge_list": [{"neighbor_idx": -1, "neighbor_name": "",
                                                         "edge_rank": states[q].shape[0], "qubit_idx": q}],
                  "side": LEFT, "batch_symbol": ""})
    mx_map = {}
    for q in qctn.qubit_indices:
        if not _has(mx, q) or mx[q] is None:
            continue
        m = mx[q]
        uid = len(L)
        mx_map[q] = uid
        bs = "a" if m.ndim == 3 else ("ab" if m.ndim == 4 else "")
        L.append({"core_idx": uid, "core_name": f"mx_{q}", "tensor_source": "mx", "tensor_key": q,
                  "in_edge_list": [{"neighbor_idx": -1, "neighbor_name": "", "edge_rank": m.shape[-2], "qubit_idx": q}],
                  "out_edge_list": [{"neighbor_idx": -1, "neighbor_name": "", "edge_rank": m.shape[-1], "qubit_idx": q}],
                  "side": MIDDLE, "batch_symbol": bs})
    right_core_map = {}
    if isinstance(right_qctn, str) and right_qctn == "symmetric":
        for info in qctn.adjacency_table:
            uid = len(L)
            right_core_map[info["core_idx"]] = uid
            L.append({"core_idx": uid, "core_name": f"{info['core_name']}_R", "tensor_source": "transpose",
                      "tensor_key": info["core_name"],
                      "in_edge_list": deepcopy(info["out_edge_list"])[::-1],
                      "out_edge_list": deepcopy(info["in_edge_list"])[::-1], "side": RIGHT, "batch_symbol": ""})
    elif isinstance(right_qctn, QCTNRef):
        for info in right_qctn.adjacency_table:
            uid = len(L)
            cores["right_" + info["core_name"]] = right_cores[info["core_name"]]
            cidx = info["core_idx"] + len(left_core_map)
            right_core_map[cidx] = uid
            L.append({"core_idx": uid, "core_name": f"{info['core_name']}_R", "tensor_source": "core",
                      "tensor_key": "right_" + info["core_name"],
                      "in_edge_list": deepcopy(info["in_edge_list"]),
                      "out_edge_list": deepcopy(info["out_edge_list"]), "side": RIGHT, "batch_symbol": ""})
    right_circuit_map = {}
    for q in qctn.qubit_indices:
        if not _has(states, q):
            continue
        uid = len(L)
        right_circuit_map[q] = uid
        L.append({"core_idx": uid, "core_name": f"circuit_R_{q}", "tensor_source": "circuit", "tensor_key": q,
                  "in_edge_list": [{"neighbor_idx": -1, "neighbor_name": "", "edge_rank": states[q].shape[0],
                                    "qubit_idx": q}],
                  "out_edge_list": [], "side": RIGHT, "batch_symbol": ""})

    # ---- Step 2 (the reference looks neighbours up in left/right_core_map by ORIGINAL index)
    for orig, nid in left_core_map.items():
        e = L[nid]
        for ed in e["in_edge_list"]:
            if ed["neighbor_idx"] == -1:
                q = ed["qubit_idx"]
                if q in left_circuit_map:
                    u = left_circuit_map[q]
                    ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
                    L[u]["out_edge_list"][0]["neighbor_idx"] = nid
                    L[u]["out_edge_list"][0]["neighbor_name"] = e["core_name"]
            elif ed["neighbor_idx"] in left_core_map:
                u = left_core_map[ed["neighbor_idx"]]
                ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
        for ed in e["out_edge_list"]:
            if ed["neighbor_idx"] == -1:
                q = ed["qubit_idx"]
                if q in mx_map:
                    u = mx_map[q]
                    ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
                    L[u]["in_edge_list"][0]["neighbor_idx"] = nid
                    L[u]["in_edge_list"][0]["neighbor_name"] = e["core_name"]
            elif ed["neighbor_idx"] in left_core_map:
                u = left_core_map[ed["neighbor_idx"]]
                ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
    for orig, nid in right_core_map.items():
        e = L[nid]
        for ed in e["in_edge_list"]:
            if ed["neighbor_idx"] == -1:
                q = ed["qubit_idx"]
                if q in mx_map:
                    u = mx_map[q]
                    ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
                    L[u]["out_edge_list"][0]["neighbor_idx"] = nid
                    L[u]["out_edge_list"][0]["neighbor_name"] = e["core_name"]
            elif ed["neighbor_idx"] in right_core_map:
                u = right_core_map[ed["neighbor_idx"]]
                ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
        for ed in e["out_edge_list"]:
            if ed["neighbor_idx"] == -1:
                q = ed["qubit_idx"]
                if q in right_circuit_map:
                    u = right_circuit_map[q]
                    ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]
                    L[u]["in_edge_list"][0]["neighbor_idx"] = nid
                    L[u]["in_edge_list"][0]["neighbor_name"] = e["core_name"]
            elif ed["neighbor_idx"] in right_core_map:
                u = right_core_map[ed["neighbor_idx"]]
                ed["neighbor_idx"], ed["neighbor_name"] = u, L[u]["core_name"]

    # ---- Step 2.5 symbols
    def gen():
        i = 0
        while True:
            s = get_symbol(i)
            if s not in ("a", "b"):
                yield s
            i += 1
    g = gen()
    for e in L:
        for ed in e["out_edge_list"]:
            if "symbol" in ed:
                continue
            ed["symbol"] = next(g)
            nb = ed["neighbor_idx"]
            if nb >= 0:
                for ie in L[nb]["in_edge_list"]:
                    if ie["neighbor_idx"] == e["core_idx"] and ie["qubit_idx"] == ed["qubit_idx"]:
                        ie["symbol"] = ed["symbol"]
                        break
    for e in L:
        for ed in e["in_edge_list"]:
            if "symbol" not in ed:
                ed["symbol"] = next(g)

    # ---- Step 3
    next_uid = len(L)
    for q in qctn.qubit_indices:
        on_q = [e for e in L if any(ed["qubit_idx"] == q for ed in e["in_edge_list"])
                or any(ed["qubit_idx"] == q for ed in e["out_edge_list"])]
        if not on_q:
            continue
        extra = []
        for e in on_q:
            for ed in e["in_edge_list"] + e["out_edge_list"]:
                nb = ed["neighbor_idx"]
                if nb >= 0:
                    cand = next((c for c in L if c["core_idx"] == nb), None)
                    if cand is not None and cand["tensor_source"] == "circuit" and \
                            not any(cand is x for x in on_q) and not any(cand is x for x in extra):
                        extra.append(cand)
        on_q.extend(extra)
        groups = _groups(on_q)
        new_entries, ids_rm, old2new = [], set(), {}
        for gi, grp in enumerate(groups):
            ne = _contract_group(grp, q, cores, states, mx)
            if ne is None or any(ne is m for m in grp):
                continue
            ne["core_idx"] = next_uid
            ne["core_name"] = f"merged_q{q}_g{gi}_{next_uid}"
            next_uid += 1
            new_entries.append(ne)
            for m in grp:
                ids_rm.add(m["core_idx"])
                old2new[m["core_idx"]] = ne
        if not new_entries:
            continue
        L = [e for e in L if e["core_idx"] not in ids_rm] + new_entries
        for e in L:
            for ed in e["in_edge_list"] + e["out_edge_list"]:
                if ed["neighbor_idx"] in old2new:
                    nn = old2new[ed["neighbor_idx"]]
                    ed["neighbor_idx"], ed["neighbor_name"] = nn["core_idx"], nn["core_name"]

    # ---- Step 4
    if len(L) == 1:
        return _get_tensor(L[0], cores, states, mx)
    if not L:
        raise RuntimeError("No tensor left after contraction")
    return _contract_remaining(L, cores, states, mx)


def _groups(entries):                                                  # :615-664
    n = len(entries)
    if n == 1:
        return [entries]
    pos = {e["core_idx"]: i for i, e in enumerate(entries)}
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for i, e in enumerate(entries):
        for ed in e["out_edge_list"] + e["in_edge_list"]:
            nb = ed["neighbor_idx"]
            if nb >= 0 and nb in pos:
                a, b = find(i), find(pos[nb])
                if a != b:
                    parent[a] = b
    out = {}
    for i in range(n):
        out.setdefault(find(i), []).append(entries[i])
    return list(out.values())


def _contract_group(group, q, cores, states, mx):                     # :690-990
    if len(group) == 1:
        e = group[0]
        if not any(ed["qubit_idx"] == q for ed in e["in_edge_list"] + e["out_edge_list"]):
            return e
    tensors, parts = [], []
    gidx = set(e["core_idx"] for e in group)
    cin, cout, batch = [], [], set()
    for e in group:
        t = _get_tensor(e, cores, states, mx)
        tensors.append(t)
        bs = e.get("batch_symbol", "")
        batch |= set(bs)
        part = bs

        def keep(ed):
            internal = ed["neighbor_idx"] >= 0 and ed["neighbor_idx"] in gidx
            return ed["neighbor_idx"] == -1 or (not internal and ed["qubit_idx"] != q)

        if e["side"] == RIGHT:
            n_in = e.get("original_in_edge_count", len(e["out_edge_list"]))
            n_out = e.get("original_out_edge_count", len(e["in_edge_list"]))
            dims = [None] * (t.ndim - len(bs))
            for k, ed in enumerate(e["out_edge_list"]):
                dims[n_in - 1 - k] = ed["symbol"]
                if keep(ed):
                    cout.append((ed["symbol"], dict(ed)))
            for k, ed in enumerate(e["in_edge_list"]):
                dims[n_in + n_out - 1 - k] = ed["symbol"]
                if keep(ed):
                    cin.append((ed["symbol"], dict(ed)))
            part += "".join(s for s in dims if s is not None)
        else:
            for ed in e["in_edge_list"]:
                part += ed["symbol"]
                if keep(ed):
                    cin.append((ed["symbol"], dict(ed)))
            for ed in e["out_edge_list"]:
                part += ed["symbol"]
                if keep(ed):
                    cout.append((ed["symbol"], dict(ed)))
        parts.append(part)
    outs, nb = [], ""
    if "a" in batch:
        outs.append("a"); nb += "a"
    if "b" in batch:
        outs.append("b"); nb += "b"
    outs += [s for s, _ in cin] + [s for s, _ in cout]
    eq = ",".join(parts) + "->" + "".join(outs)
    smap = {"a": "a", "b": "b", ",": ",", "-": "-", ">": ">"}
    idx = 2
    for ch in eq:
        if ch not in smap:
            smap[ch] = get_symbol(idx)
            idx += 1
    eq = "".join(smap.get(c, c) for c in eq)
    res = np.einsum(eq, *tensors)
    return {"core_idx": -1 - q, "core_name": f"merged_{q}", "tensor": res, "tensor_source": "merged",
            "tensor_key": None, "in_edge_list": [ed for _, ed in cin], "out_edge_list": [ed for _, ed in cout],
            "side": MIDDLE, "batch_symbol": nb}


def _contract_remaining(L, cores, states, mx):                        # :993-1080
    tensors = [_get_tensor(e, cores, states, mx) for e in L]
    parts, outs = [], []
    for e, t in zip(L, tensors):
        part = ""
        if e["side"] == MIDDLE:
            bd = t.ndim - 2
            if bd >= 1:
                part += "a"
            if bd >= 2:
                part += "b"
            if e["in_edge_list"]:
                part += e["in_edge_list"][0]["symbol"]
            if e["out_edge_list"]:
                part += e["out_edge_list"][0]["symbol"]
        elif e["side"] == RIGHT:
            n_in = e.get("original_in_edge_count", len(e["out_edge_list"]))
            n_out = e.get("original_out_edge_count", len(e["in_edge_list"]))
            dims = [None] * t.ndim
            for k, ed in enumerate(e["out_edge_list"]):
                dims[n_in - 1 - k] = ed["symbol"]
            for k, ed in enumerate(e["in_edge_list"]):
                dims[n_in + n_out - 1 - k] = ed["symbol"]
            part = "".join(s for s in dims if s is not None)
        else:
            for ed in e["in_edge_list"]:
                part += ed["symbol"]
            for ed in e["out_edge_list"]:
                part += ed["symbol"]
            if e.get("tensor_source") == "merged":
                extra = t.ndim - (len(e["in_edge_list"]) + len(e["out_edge_list"]))
                part = ("a" if extra >= 1 else "") + ("b" if extra >= 2 else "") + part
        parts.append(part)
        if "a" in part and "a" not in outs:
            outs.append("a")
        if "b" in part and "b" not in outs:
            outs.append("b")
    return np.einsum(",".join(parts) + "->" + "".join(outs), *tensors)
