"""Named-node DAG built from S-expression graph definitions (reference ``utilities/graph.py``).

``Graph.traverse(["(A (B D) (C D))"])`` returns the head nodes and each node's ordered
successors; optional ``(key: value)`` property lists after a successor are reported through
``node_properties_callback(successor, properties, predecessor)`` (used for the pipeline's
input/output name mapping).  ``get_path(head)`` yields the execution order — a DFS in which a
re-visited node moves to the end, i.e. a valid topological order for a DAG — and the result is
cached per head until the graph changes (the reference recomputes it every frame).
"""
from __future__ import annotations

from collections import OrderedDict

from .sexpr import parse

__all__ = ["Graph", "Node"]


class Node:
    def __init__(self, name, element=None, successors=None):
        self._name = name
        self._element = element
        self._successors = successors if successors else OrderedDict()
        self.predecessors = OrderedDict()

    def add(self, successor):
        if successor not in self._successors:
            self._successors[successor] = successor

    def remove(self, successor):
        self._successors.pop(successor, None)

    @property
    def element(self):
        return self._element

    @element.setter
    def element(self, value):
        self._element = value

    @property
    def name(self):
        return self._name

    @property
    def successors(self):
        return self._successors

    def __repr__(self):
        return f"{self._name}: {list(self._successors)}"


class Graph:
    def __init__(self, head_nodes=None):
        self._graph: "OrderedDict[str, Node]" = OrderedDict()
        self._head_nodes = head_nodes if head_nodes else OrderedDict()
        self._path_cache: dict = {}

    def __iter__(self):
        return self.get_path()

    def __repr__(self):
        return str(self.nodes(as_strings=True))

    def __len__(self):
        return len(self._graph)

    def add(self, node: Node):
        if node.name in self._graph:
            raise KeyError(f"Graph already contains node: {node}")
        self._graph[node.name] = node
        self._path_cache.clear()

    def remove(self, node: Node):
        if node.name in self._graph:
            del self._graph[node.name]
            self._path_cache.clear()

    def get_node(self, node_name) -> Node:
        return self._graph[node_name]

    @property
    def head_nodes(self):
        return self._head_nodes

    def _execution_order(self, head_node_name):
        ordered: "OrderedDict[Node, None]" = OrderedDict()
        if not self._head_nodes:
            return []
        if not head_node_name:
            head_node_name = next(iter(self._head_nodes))
        if head_node_name not in self._head_nodes:
            return []
        # iterative DFS reproducing "move re-visited node to the end"
        stack = [self._graph[head_node_name]]
        while stack:
            node = stack.pop()
            if node in ordered:
                del ordered[node]
            ordered[node] = None
            for succ in reversed(list(node.successors)):
                stack.append(self._graph[succ])
        return list(ordered)

    def get_path(self, head_node_name=None):
        key = head_node_name
        path = self._path_cache.get(key)
        if path is None:
            path = self._execution_order(head_node_name)
            self._path_cache[key] = path
        return iter(path)

    def invalidate(self):
        self._path_cache.clear()

    def iterate_after(self, node_name, head_node_name=None):
        ordered = list(self.get_path(head_node_name))
        node = self.get_node(node_name)
        try:
            return ordered[ordered.index(node) + 1:]
        except ValueError:
            return []

    def nodes(self, as_strings=False):
        return [n.name if as_strings else n for n in self._graph.values()]

    @classmethod
    def path_local(cls, graph_path):
        """``"local:remote"`` -> ``"local"`` (None when empty)."""
        if isinstance(graph_path, str):
            graph_path = graph_path.partition(":")[0] or None
        return graph_path

    @classmethod
    def path_remote(cls, graph_path):
        """``"local:remote"`` -> ``"remote"`` (None when empty)."""
        if isinstance(graph_path, str):
            graph_path = graph_path.partition(":")[2] or None
        return graph_path

    @classmethod
    def traverse(cls, graph_definition, node_properties_callback=None):
        heads: "OrderedDict[str, str]" = OrderedDict()
        successors: "OrderedDict[str, OrderedDict]" = OrderedDict()

        def add_successor(node, succ):
            if isinstance(node, dict):
                return
            table = successors.setdefault(node, OrderedDict())
            if isinstance(succ, str):
                table[succ] = succ
            elif succ and isinstance(succ, dict) and node_properties_callback and table:
                node_properties_callback(next(reversed(table)), succ, node)

        def walk(node, succs):
            for succ in succs:
                if isinstance(succ, list):
                    add_successor(node, succ[0])
                    walk(succ[0], succ[1:])
                else:
                    add_successor(node, succ)
                    add_successor(succ, None)

        for subgraph in graph_definition:
            node, succs = parse(subgraph)
            heads[node] = node
            add_successor(node, None)
            walk(node, succs)
        return heads, successors
