"""``ByzantineRandomizedConsensus`` (reference: core/byzantinerandomizedconsensus.py:10-106).

The round logic -- the BRB deliver upcall, ``get_max_val`` and the phase/round advance
(:53-106) -- runs inside the HIP engine for every replica of the peer list at once; this class
keeps the reference's constructor (note the argument order: ``peer_list`` before
``host_address``), ``message_queue``, ``start``/``propose`` and the ``decide`` upcall to
``consensus_user`` (:94).
"""
import json
import queue

from ..base.broadcast import IBroadcastHandler
from ..base.consensus import Consensus
from .brbroadcast import BRBroadcast


class ByzantineRandomizedConsensus(Consensus, IBroadcastHandler):
    NONE = -1
    PHASE1 = 1
    PHASE2 = 2

    def __init__(self, total_nodes, faulty_nodes, peer_list, host_address, consensus_user):
        assert total_nodes > 5 * faulty_nodes, "Number of nodes doesn't satisfy N>5f assumption"   # :20
        self.message_queue = queue.Queue(20)
        self.N = total_nodes
        self.f = faulty_nodes
        self.round = 0
        self.phase = 0
        self.brb = BRBroadcast(total_nodes, faulty_nodes, host_address, peer_list, self)
        self.consensus_user = consensus_user
        self.brb.cluster.add_consensus(self, self.brb.node_id)
        self.brb.broadcast_listener()
        self.host_address = host_address

    def start(self):
        proposal = self.message_queue.get_nowait()
        print("Consensus started on " + str(self.host_address))
        self.propose(proposal)

    def propose(self, message):
        self.round = 1
        self.phase = 1
        self.brb.cluster.propose(self.brb.node_id, str(message))
        print("Proposal sent on " + str(self.host_address))

    def deliver(self, message):
        """The IBroadcastHandler upcall (:53).  BRB deliveries of the cluster's own traffic are
        consumed inside the engine; a direct call -- a JSON message as the reference builds it
        (:48-49), {"host": address, "round": r, "phase": p, "message": value} -- is handed to this
        replica's consensus state at the cluster's current step (round and phase are not read,
        as in the reference).  A non-string "message" or a host outside the peer list raises
        EngineError (network.py's deviation notes)."""
        d = json.loads(message)
        self.brb.cluster.deliver(self.brb.node_id, tuple(d["host"]), d["message"])
