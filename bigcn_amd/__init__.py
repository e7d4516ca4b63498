"""bigcn_amd - MI355X-native (gfx950) BiGCN bidirectional message-passing path.

Drop-in symbols for the reference's hot path (cwkd/BiGCN):

* ``GCNConv``       <- ``from torch_geometric.nn import GCNConv``   (BiGCN_Twitter.py:15)
* ``scatter_mean``  <- ``from torch_scatter import scatter_mean``   (BiGCN_Twitter.py:6)
* ``TDrumorGCN``, ``BUrumorGCN``, ``BiGCN`` (Twitter, 4 classes), ``Net`` (Weibo, 2 classes)
* ``FusedTrainStep`` - the training-loop body (BiGCN_Twitter.py:183-189) as one native call
  + the data-parallel all-reduce + fused Adam

all backed by hand-written HIP kernels in ``libbgcn.so`` (C ABI: ``include/bgcn.h``).
"""
from .bigcn import BiGCN, BUrumorGCN, Net, TDrumorGCN, make_optimizer
from .conv import GCNConv
from .ops import Graph, bigcn_encoder, build_graph, gcn_conv, scatter_mean, spmm
from .optim import FusedAdam, bigcn_adam
from .train import FusedTrainStep

__all__ = ["GCNConv", "scatter_mean", "TDrumorGCN", "BUrumorGCN", "BiGCN", "Net", "make_optimizer",
           "Graph", "build_graph", "gcn_conv", "spmm", "bigcn_encoder", "FusedAdam", "bigcn_adam",
           "FusedTrainStep"]
__version__ = "0.1.0"
