"""Tree and alignment readers that reproduce DendroPy's ordering (no dendropy).

The reference reads its inputs with DendroPy (``phylostan/phylostan.py:165-
191``): the tree first, ``rooting='force-rooted'``, ``preserve_underscores=
True``; then the alignment into the SAME taxon namespace, so the namespace
order -- and therefore the tip numbering of ``utils.setup_indexes`` -- is the
order in which leaves first appear in the tree file (or the TAXLABELS order
of a NEXUS tree file).  DendroPy itself is not available here; this module
restates the parts of its behaviour the data layout depends on:

* Newick: children kept in file order; ``[...]`` comments skipped; quoted
  labels unquoted; underscores preserved; branch lengths parsed as float.
* ``postorder_node_iter`` (children in order, then the node) and
  ``preorder_node_iter`` (node, then children in order).
* ``resolve_polytomies()``: a node with k > 2 children keeps its first child
  and the remaining ones are joined pairwise from the end under new
  zero-length nodes.  DendroPy's exact tie order is not available here
  (dependency absent, version unpinned in ``setup.py:28``): the likelihood is
  invariant to it, only internal node numbering could differ -- documented as
  parity-unpinned in DESIGN.md.
* ``reroot_at_edge(edge)`` (what ``phylostan parse`` does to a root with more
  than two children, ``phylostan.py:140-141``): DendroPy 4's algorithm -- a
  new node is appended to the edge's tail, the head moves under it, and the
  tree is reseeded there, so the new root's children are [head, old root]
  and the old root keeps its other children in order.  For a trifurcating
  root (A, B, C) that is (A, (B, C)): the shape -- and node numbering --
  ``resolve_polytomies`` gives ``run``.
"""
import re


class Node:
    def __init__(self, label=None, edge_length=None):
        self.label = label
        self.edge_length = edge_length
        self.parent_node = None
        self._children = []
        self.taxon = None
        self.index = -1
        self.date = 0.0
        self.annotations = _Annotations()

    # DendroPy-compatible accessors used by the reference's utils
    def child_node_iter(self):
        return iter(list(self._children))

    def child_nodes(self):
        return list(self._children)

    def is_leaf(self):
        return not self._children

    def is_internal(self):
        return bool(self._children)

    def add_child(self, node):
        node.parent_node = self
        self._children.append(node)
        return node

    def remove_child(self, node):
        self._children.remove(node)
        node.parent_node = None
        return node

    @property
    def edge(self):
        return _Edge(self)

    def postorder_iter(self):
        stack = [(self, False)]
        while stack:
            node, done = stack.pop()
            if done or not node._children:
                yield node
            else:
                stack.append((node, True))
                for ch in reversed(node._children):
                    stack.append((ch, False))

    def preorder_iter(self):
        stack = [self]
        while stack:
            node = stack.pop()
            yield node
            for ch in reversed(node._children):
                stack.append(ch)


class _Edge:
    def __init__(self, node):
        self._node = node

    @property
    def length(self):
        return self._node.edge_length

    @length.setter
    def length(self, v):
        self._node.edge_length = v


class _Annotations:
    def add_bound_attribute(self, name):
        pass


class Taxon:
    __slots__ = ("label",)

    def __init__(self, label):
        self.label = label

    def __str__(self):
        # DendroPy quotes labels containing spaces; the reference strips "'".
        return "'%s'" % self.label if " " in self.label else self.label

    def __repr__(self):
        return "Taxon(%r)" % self.label


class Tree:
    def __init__(self, seed_node, taxon_namespace):
        self.seed_node = seed_node
        self.taxon_namespace = taxon_namespace

    def postorder_node_iter(self):
        return self.seed_node.postorder_iter()

    def preorder_node_iter(self):
        return self.seed_node.preorder_iter()

    def leaf_node_iter(self):
        return (n for n in self.seed_node.preorder_iter() if n.is_leaf())

    def reroot_at_edge(self, edge, length1=None, length2=None, update_bipartitions=False):
        """DendroPy's ``Tree.reroot_at_edge`` for an edge below the current
        root (the only use: ``phylostan.py:141``).  The split edge's two
        pieces get ``length1`` (new root -> old root) and ``length2`` (new
        root -> head)."""
        head = edge._node
        tail = head.parent_node
        if tail is None or tail is not self.seed_node:
            raise ValueError("reroot_at_edge: only edges below the root are supported")
        new_seed = Node(edge_length=length1)
        tail.add_child(new_seed)
        tail.remove_child(head)
        new_seed.add_child(head)
        head.edge_length = length2
        # reseed: the old root becomes the last child of the new seed
        tail.remove_child(new_seed)
        tail.edge_length = new_seed.edge_length
        new_seed.edge_length = None
        new_seed.add_child(tail)
        self.seed_node = new_seed

    def adjacent_nodes(self):
        return self.seed_node.child_nodes()

    def resolve_polytomies(self, limit=2, update_bipartitions=False):
        polytomies = [n for n in self.postorder_node_iter() if len(n._children) > limit]
        for node in polytomies:
            while len(node._children) > limit:
                nn1 = node._children[-2]
                nn2 = node._children[-1]
                node.remove_child(nn1)
                node.remove_child(nn2)
                nn = Node(edge_length=0.0)
                nn.add_child(nn1)
                nn.add_child(nn2)
                node.add_child(nn)

    def num_taxa(self):
        return len(self.taxon_namespace)


_TOKEN = re.compile(r"\s*(\[[^\]]*\]|'(?:[^']|'')*'|[(),:;]|[^\s(),:;\[\]']+)")


def parse_newick(text, taxon_namespace=None, translate=None):
    """Parse one Newick tree string.  ``taxon_namespace`` (a list of Taxon) is
    extended in order of first appearance; ``translate`` maps NEXUS
    TRANSLATE tokens to labels."""
    if taxon_namespace is None:
        taxon_namespace = []
    by_label = {t.label: t for t in taxon_namespace}
    pos = 0
    tokens = []
    text = text.strip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ValueError("bad Newick near %r" % text[pos:pos + 30])
        tok = m.group(1)
        pos = m.end()
        if tok.startswith("["):
            continue  # comment / annotation
        tokens.append(tok)
    root = None
    stack = []  # open internal nodes
    last = None  # node that a following label / ":length" applies to
    i = 0
    while i < len(tokens):
        tok = tokens[i]
        if tok == "(":
            node = Node()
            if stack:
                stack[-1].add_child(node)
            else:
                root = node
            stack.append(node)
            last = None
        elif tok == ",":
            last = None
        elif tok == ")":
            last = stack.pop()
        elif tok == ":":
            i += 1
            last.edge_length = float(tokens[i])
        elif tok == ";":
            break
        else:
            label = tok
            if label.startswith("'"):
                label = label[1:-1].replace("''", "'")
            if last is None:
                leaf = Node(label)
                if stack:
                    stack[-1].add_child(leaf)
                else:
                    root = leaf
                last = leaf
            else:
                last.label = label
        i += 1
    for node in root.preorder_iter():
        if node.is_leaf():
            label = node.label
            if translate and label in translate:
                label = translate[label]
            if label not in by_label:
                t = Taxon(label)
                by_label[label] = t
                taxon_namespace.append(t)
            node.taxon = by_label[label]
    return Tree(root, taxon_namespace)


def _nexus_blocks(text):
    blocks = {}
    for m in re.finditer(r"begin\s+(\w+)\s*;(.*?)\bend\s*;", text, re.S | re.I):
        blocks.setdefault(m.group(1).lower(), []).append(m.group(2))
    return blocks


def _strip_nexus_comments(text):
    return re.sub(r"\[[^\]]*\]", "", text)


def read_tree(path, tree_offset=0):
    """Read the first (``tree_offset``) tree of a Newick or NEXUS file the way
    ``Tree.get(..., rooting='force-rooted', preserve_underscores=True)`` does
    in ``phylostan.py:167-173``."""
    with open(path) as fp:
        text = fp.read()
    if text.lstrip().upper().startswith("#NEXUS"):
        blocks = _nexus_blocks(text)
        namespace = []
        for tb in blocks.get("taxa", []):
            m = re.search(r"taxlabels(.*?);", _strip_nexus_comments(tb), re.S | re.I)
            if m:
                for lab in m.group(1).split():
                    namespace.append(Taxon(lab.strip("'")))
        trees = []
        translate = {}
        for tb in blocks.get("trees", []):
            m = re.search(r"translate(.*?);", tb, re.S | re.I)
            if m:
                for entry in m.group(1).split(","):
                    parts = entry.split()
                    if len(parts) >= 2:
                        translate[parts[0]] = parts[1].strip("'")
            for tm in re.finditer(r"tree\s+[^=]+=\s*(?:\[&[RrUu]\]\s*)?(.*?;)", tb, re.S | re.I):
                trees.append(tm.group(1))
        return parse_newick(trees[tree_offset], namespace, translate or None)
    lines = [ln for ln in text.split(";") if ln.strip()]
    return parse_newick(lines[tree_offset] + ";")


def read_alignment(path):
    """Read a FASTA or NEXUS DNA alignment -> ordered dict label -> sequence
    (upper case).  FASTA is detected as in ``phylostan.py:186-189``."""
    with open(path) as fp:
        text = fp.read()
    seqs = {}
    if text.lstrip().startswith(">"):
        name = None
        for line in text.splitlines():
            line = line.strip()
            if not line:
                continue
            if line.startswith(">"):
                name = line[1:].strip()
                seqs[name] = []
            else:
                seqs[name].append(line)
        return {k: "".join(v).upper() for k, v in seqs.items()}
    blocks = _nexus_blocks(text)
    body = (blocks.get("data") or blocks.get("characters"))[0]
    body = _strip_nexus_comments(body)
    m = re.search(r"matrix(.*)", body, re.S | re.I)
    mat = m.group(1).rsplit(";", 1)[0] if ";" in m.group(1) else m.group(1)
    order = []
    for line in mat.splitlines():
        parts = line.split()
        if len(parts) < 2:
            continue
        name = parts[0].strip("'")
        if name not in seqs:
            seqs[name] = []
            order.append(name)
        seqs[name].append("".join(parts[1:]))
    return {k: "".join(seqs[k]).upper() for k in order}
