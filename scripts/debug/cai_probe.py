import torch
x = torch.arange(10, dtype=torch.int64, device="cuda")
class V:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}
y = torch.as_tensor(V(x.data_ptr() + 16, 4), device="cuda")
print("view", y, y.data_ptr() == x.data_ptr() + 16)
y += 100
print(x)
