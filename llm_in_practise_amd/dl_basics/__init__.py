"""Deep-learning basics track (``DL_Basics/ANN_Basics.ipynb`` and ``DL_Basics/CNN_and_RNN.ipynb``).

The reference teaches these in notebooks; here they are importable, tested modules:

* :mod:`.numpy_nn`   — NumPy MLPs with hand-written backprop, losses, L2 regularisation,
  mini-batch training and the SGD / Momentum / AdaGrad / RMSProp / Adam optimisers;
* :mod:`.numpy_rnn`  — manual RNN / LSTM / GRU forward passes and BPTT in PyTorch's gate layout
  (checked against ``torch.nn.RNN/LSTM/GRU`` and autograd);
* :mod:`.numpy_cnn`  — conv2d / max-pool forward + backward (sliding-window einsum), LeNet-5;
* :mod:`.embeddings` — random / GloVe-initialised ``nn.Embedding`` (frozen or trainable);
* :mod:`.seq2seq`    — GRU encoder / Bahdanau-attention decoder with teacher forcing and greedy
  decoding, plus the variable-length ``pad_collate`` used with ``DataLoader``.
"""
from .numpy_nn import MLP, Adam, AdaGrad, Momentum, RMSProp, SGD, train_mlp  # noqa: F401
