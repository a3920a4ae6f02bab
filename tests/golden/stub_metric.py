"""Stand-ins for the FID pipeline's two networks (test infrastructure): the Inception detector (a pickle on NGC
that cannot be fetched here) and a generator that runs on the CPU.  Both are deterministic functions of their
inputs, so the reference's metric code (SG3/metrics/metric_utils.py:201-306, frechet_inception_distance.py:19-40)
and this build's give comparable statistics when they see the same images, labels and latents."""
import torch


class StubDetector(torch.nn.Module):
    """images [N, 3, H, W] (uint8, or float [0, 255] where the reference's real-image path passes them through)
    -> features [N, F] float32: a fixed random projection of the 4 x 4 average-pooled image plus its square."""

    def __init__(self, res=16, num_features=8, seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        k = 3 * (res // 4) ** 2
        self.register_buffer('P', torch.randn([2 * k, num_features], generator=g, dtype=torch.float64) / k)

    def forward(self, x, return_features=True):
        assert return_features
        x = torch.nn.functional.avg_pool2d(x.to(torch.float64) / 255, 4).flatten(1)
        return (torch.cat([x, x.square()], 1) @ self.P).to(torch.float32)


class StubGenerator(torch.nn.Module):
    """z [N, z_dim], c [N, c_dim] -> images [N, C, res, res] in about [-1.1, 1.1] (so the uint8 clamp matters)."""

    def __init__(self, z_dim=8, c_dim=2, img_channels=2, res=16, seed=1):
        super().__init__()
        self.z_dim, self.c_dim, self.img_channels, self.img_resolution = z_dim, c_dim, img_channels, res
        g = torch.Generator().manual_seed(seed)
        self.register_buffer('A', torch.randn([z_dim + c_dim, img_channels * res * res], generator=g) / (z_dim ** 0.5))

    def forward(self, z, c, **kwargs):
        h = torch.cat([z, c.to(z.dtype)], 1) if self.c_dim else z
        return (torch.tanh(h @ self.A) * 1.1).reshape(-1, self.img_channels, self.img_resolution, self.img_resolution)
