"""``Broadcast`` / ``IBroadcastHandler`` (reference: base/broadcast.py:5-55).

Same constructor, attributes and method signatures as the reference.  ``broadcast()`` hands the
message to the node's simulated cluster instead of opening one TCP connection per peer
(base/broadcast.py:26-40); the JSON envelope ``{"peer", "type", "message"}`` (:37) is not
materialised because nothing reads it off a wire.
"""
from abc import ABCMeta, abstractmethod


class Broadcast(metaclass=ABCMeta):
    """A broadcast protocol endpoint: ``host`` is this node's address, ``peers`` every node's
    address, self included (base/broadcast.py:13-15, :30)."""

    BUFFER_SIZE = 1024   # base/broadcast.py:11 (kept for API compatibility; no sockets here)

    def __init__(self, host_address, peer_list):
        self.host = host_address
        self.peers = peer_list

    def broadcast(self, message_type, message):
        """Send ``message`` of ``message_type`` to every peer, self included."""
        self._cluster_send(message_type, message)

    def _cluster_send(self, message_type, message):
        raise NotImplementedError("%s has no simulated transport" % type(self).__name__)

    @abstractmethod
    def broadcast_listener(self):
        pass


class IBroadcastHandler(metaclass=ABCMeta):
    """The DELIVER upcall of a broadcast protocol (base/broadcast.py:47-55)."""

    @abstractmethod
    def deliver(self, message):
        pass
