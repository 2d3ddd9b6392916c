import torch.nn as nn
import torch.nn.functional as F


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        h, g = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(g)


class FeedForward(nn.Module):
    def __init__(self, dim, dim_out=None, mult=4, dropout=0.0, activation_fn="geglu", **kw):
        super().__init__()
        inner = int(dim * mult)
        dim_out = dim_out if dim_out is not None else dim
        assert activation_fn == "geglu"
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim_out)])

    def forward(self, x):
        for m in self.net:
            x = m(x)
        return x


class AdaLayerNorm(nn.Module):
    def __init__(self, *a, **k):
        raise NotImplementedError
