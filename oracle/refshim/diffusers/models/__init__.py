import torch.nn as nn


class ModelMixin(nn.Module):
    @property
    def config(self):
        return self._internal_dict

    @property
    def dtype(self):
        return next(self.parameters()).dtype
