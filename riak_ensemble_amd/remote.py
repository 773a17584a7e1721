"""Streaming exchange with a tree owned by another process.

The reference drives a remote tree through a fun:
``Remote(start_exchange_level, {Level, Buckets})`` once per level, then
``Remote(exchange_get, {Level, Bucket})`` per bucket (src/synctree.erl:397-417).
In riak_ensemble every ``exchange_get`` is a ``gen_server:call`` to the peer
tree (src/riak_ensemble_exchange.erl:72-81, riak_ensemble_peer_tree.erl:
155-157); test/synctree_remote.erl:25-66 streams a level instead: the remote
process answers ``start_exchange_level`` and pushes every bucket of the level.

Here the remote side is a process that owns a device tree (:func:`serve`).
A level is ONE request and ONE reply: the server answers
``start_exchange_level`` with the node images of every requested bucket from a
single batched device call (``exchange_get_batch``: path verification and the
images for the whole level on the GPU), and the client's fun
(:class:`RemoteTree`.fun) serves the level's ``exchange_get`` calls from that
reply.  A bucket that was not announced falls back to a single request, as the
reference's remote fun does (``after 0 -> Other ! {get_bucket, ...}``).

Wire format: Erlang external term format (``terms.term_to_binary``) of
``{start_exchange_level, Level, Buckets}`` / ``{exchange_get, Level, Bucket}``
/ ``stop`` requests and of the replies -- the images the reference's
``send_bucket`` sends (``term_to_binary(Reply)``), so the byte counts
(:attr:`RemoteTree.stats`) are comparable with test/synctree_remote.erl's.
"""
import multiprocessing as mp

from . import synctree
from . import terms


def _images(tree, level, buckets):
    return synctree.exchange_get_batch(level, list(buckets), tree)


def serve(conn, factory, args=()):
    """Server loop: build the tree with ``factory(*args)`` (a synctree tree
    record, or any object with ``exchange_get_batch(level, buckets)``), then
    answer requests on ``conn`` until ``stop``.  Runs in the remote process."""
    tree = factory(*args)
    get = tree.exchange_get_batch if hasattr(tree, 'exchange_get_batch') else (lambda l, b: _images(tree, l, b))
    msgs = nbytes = 0
    conn.send_bytes(terms.term_to_binary('ready'))
    while True:
        req = terms.binary_to_term(conn.recv_bytes())
        if req == 'stop':
            conn.send_bytes(terms.term_to_binary(('stats', msgs, nbytes)))
            return
        op = req[0]
        if op == 'start_exchange_level':
            _, level, buckets = req
            reply = terms.term_to_binary(('level', level, list(get(level, list(buckets)))))
        elif op == 'exchange_get':
            _, level, bucket = req
            reply = terms.term_to_binary(('bucket', get(level, [bucket])[0]))
        else:
            reply = terms.term_to_binary(('error', 'badarg'))
        msgs += 1
        nbytes += len(reply)
        conn.send_bytes(reply)


class RemoteTree:
    """Client side: a process owning the remote tree and the remote fun.

    ``factory`` builds the remote tree inside the child process (it must be
    importable there: a module-level function).  Use as a context manager."""

    def __init__(self, factory, args=(), start_method='spawn'):
        ctx = mp.get_context(start_method)
        self._conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=serve, args=(child, factory, args), daemon=True)
        self.proc.start()
        child.close()
        if terms.binary_to_term(self._conn.recv_bytes()) != 'ready':
            raise RuntimeError('remote tree did not start')
        self._cache = {}
        self.requests = 0          # messages this side sent
        self.levels = []           # (level, buckets) announced
        self.stats = None          # server's (messages, reply bytes) after close()

    def _call(self, req):
        self.requests += 1
        self._conn.send_bytes(terms.term_to_binary(req))
        return terms.binary_to_term(self._conn.recv_bytes())

    def fun(self, op, arg):
        """The remote fun of synctree:compare/3 (synctree.erl:397-417)."""
        if op == 'start_exchange_level':
            level, buckets = arg
            rep = self._call(('start_exchange_level', level, list(buckets)))
            self._cache = {(level, b): img for b, img in zip(buckets, rep[2])}
            self.levels.append((level, len(buckets)))
            return 'ok'
        if op == 'exchange_get':
            img = self._cache.pop(tuple(arg), None)
            if img is None:   # not streamed: one request for this bucket
                img = self._call(('exchange_get', arg[0], arg[1]))[1]
            return img
        raise ValueError('function_clause: remote fun %r' % (op,))

    def close(self):
        if self.proc is not None:
            rep = self._call('stop')
            self.stats = (rep[1], rep[2])
            self.proc.join(timeout=60)
            self.proc = None
            self._conn.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        try:
            self.close()
        finally:
            if self.proc is not None and self.proc.is_alive():
                self.proc.kill()
