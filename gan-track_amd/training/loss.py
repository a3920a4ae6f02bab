"""StyleGAN2-ADA loss: non-saturating logistic loss, style mixing, path-length (Greg) and R1 (Dreg)
regularisers.  Drop-in for SG3/training/loss.py:17-139 (same class, constructor arguments, phase
names and reported statistics).

The second-order passes run on the HIP kernels: Greg differentiates through
autograd.grad(create_graph=True) of the generator (modulated conv = conv / transposed conv / wgrad,
upfirdn2d, bias_act grad-of-grad), Dreg through D and the ADA warp (grid_sample backward-of-backward).
"""
import numpy as np
import torch

from torch_utils import training_stats
from torch_utils.ops import conv2d_gradfix
from torch_utils.ops import upfirdn2d


class Loss:
    def accumulate_gradients(self, phase, real_img, real_c, gen_z, gen_c, gain, cur_nimg):
        raise NotImplementedError()


class StyleGAN2Loss(Loss):
    def __init__(self, device, G, D, augment_pipe=None, r1_gamma=10, style_mixing_prob=0, pl_weight=0,
                 pl_batch_shrink=2, pl_decay=0.01, pl_no_weight_grad=False, blur_init_sigma=0, blur_fade_kimg=0,
                 allow_aug_debug_print=False):
        super().__init__()
        self.device = device
        self.G, self.D, self.augment_pipe = G, D, augment_pipe
        self.r1_gamma = r1_gamma
        self.style_mixing_prob = style_mixing_prob
        self.pl_weight, self.pl_batch_shrink, self.pl_decay = pl_weight, pl_batch_shrink, pl_decay
        self.pl_no_weight_grad = pl_no_weight_grad
        self.pl_mean = torch.zeros([], device=device)
        self.blur_init_sigma, self.blur_fade_kimg = blur_init_sigma, blur_fade_kimg
        self.allow_aug_debug_print = allow_aug_debug_print

    def run_G(self, z, c, update_emas=False):
        if self.style_mixing_prob <= 0:
            ws = self.G.mapping(z, c, update_emas=update_emas)
            return self.G.synthesis(ws, update_emas=update_emas), ws
        with torch.autograd.profiler.record_function('style_mixing'):
            # the draws of loss.py:45-49 in their order (the first mapping draws nothing), then ONE batched
            # mapping pass over [z; z2] instead of two: the mapping is row-independent, and this halves its
            # ~75 launches (forward + backward) per G pass.  The w_avg EMA (update_emas) sees z's rows only.
            cutoff = torch.empty([], dtype=torch.int64, device=z.device).random_(1, self.G.num_ws)
            cutoff = torch.where(torch.rand([], device=z.device) < self.style_mixing_prob, cutoff,
                                 torch.full_like(cutoff, self.G.num_ws))
            z2 = torch.randn_like(z)
            n = z.shape[0]
            ws_all = self.G.mapping(torch.cat([z, z2]), torch.cat([c, c]), update_emas=False)
            ws, ws2 = ws_all[:n], ws_all[n:]
            m = self.G.mapping
            if update_emas and getattr(m, 'w_avg_beta', None) is not None:
                m.w_avg.copy_(ws[:, 0].detach().mean(dim=0).lerp(m.w_avg, m.w_avg_beta))
            # ws[:, cutoff:] = ws2[:, cutoff:] as a device-side select: slicing by a device tensor would read
            # it back to the host (a sync per call, and no HIP-graph capture)
            mix = (torch.arange(ws.shape[1], device=ws.device) >= cutoff).reshape(1, -1, 1)
            ws = torch.where(mix, ws2, ws)
        img = self.G.synthesis(ws, update_emas=update_emas)
        return img, ws

    def run_D(self, img, c, blur_sigma=0, update_emas=False, allow_aug_debug_print=False):
        blur_size = np.floor(blur_sigma * 3)
        if blur_size > 0:
            with torch.autograd.profiler.record_function('blur'):
                f = torch.arange(-blur_size, blur_size + 1, device=img.device).div(blur_sigma).square().neg().exp2()
                img = upfirdn2d.filter2d(img, f / f.sum())
        if self.augment_pipe is not None:
            img = self.augment_pipe(img, allow_aug_debug_print)
        return self.D(img, c, update_emas=update_emas)

    def accumulate_gradients(self, phase, real_img, real_c, gen_z, gen_c, gain, cur_nimg):
        assert phase in ['Gmain', 'Greg', 'Gboth', 'Dmain', 'Dreg', 'Dboth']
        if self.pl_weight == 0:
            phase = {'Greg': 'none', 'Gboth': 'Gmain'}.get(phase, phase)
        if self.r1_gamma == 0:
            phase = {'Dreg': 'none', 'Dboth': 'Dmain'}.get(phase, phase)
        blur_sigma = max(1 - cur_nimg / (self.blur_fade_kimg * 1e3), 0) * self.blur_init_sigma \
            if self.blur_fade_kimg > 0 else 0
        report = training_stats.report

        if phase in ['Gmain', 'Gboth']:
            with torch.autograd.profiler.record_function('Gmain_forward'):
                gen_img, _ = self.run_G(gen_z, gen_c)
                logits = self.run_D(gen_img, gen_c, blur_sigma=blur_sigma)
                report('Loss/scores/fake', logits)
                report('Loss/signs/fake', logits.sign())
                loss_G = torch.nn.functional.softplus(-logits)
                report('Loss/G/loss', loss_G)
            with torch.autograd.profiler.record_function('Gmain_backward'):
                loss_G.mean().mul(gain).backward()

        if phase in ['Greg', 'Gboth']:
            with torch.autograd.profiler.record_function('Gpl_forward'):
                bs = gen_z.shape[0] // self.pl_batch_shrink
                gen_img, gen_ws = self.run_G(gen_z[:bs], gen_c[:bs])
                pl_noise = torch.randn_like(gen_img) / np.sqrt(gen_img.shape[2] * gen_img.shape[3])
                with torch.autograd.profiler.record_function('pl_grads'), \
                        conv2d_gradfix.no_weight_gradients(self.pl_no_weight_grad):
                    pl_grads = torch.autograd.grad(outputs=[(gen_img * pl_noise).sum()], inputs=[gen_ws],
                                                   create_graph=True, only_inputs=True)[0]
                pl_lengths = pl_grads.square().sum(2).mean(1).sqrt()
                pl_mean = self.pl_mean.lerp(pl_lengths.mean(), self.pl_decay)
                self.pl_mean.copy_(pl_mean.detach())
                pl_penalty = (pl_lengths - pl_mean).square()
                report('Loss/pl_penalty', pl_penalty)
                loss_Gpl = pl_penalty * self.pl_weight
                report('Loss/G/reg', loss_Gpl)
            with torch.autograd.profiler.record_function('Gpl_backward'):
                loss_Gpl.mean().mul(gain).backward()

        loss_Dgen = 0
        if phase in ['Dmain', 'Dboth']:
            with torch.autograd.profiler.record_function('Dgen_forward'):
                gen_img, _ = self.run_G(gen_z, gen_c, update_emas=True)
                logits = self.run_D(gen_img, gen_c, blur_sigma=blur_sigma, update_emas=True)
                report('Loss/scores/fake', logits)
                report('Loss/signs/fake', logits.sign())
                loss_Dgen = torch.nn.functional.softplus(logits)
            with torch.autograd.profiler.record_function('Dgen_backward'):
                loss_Dgen.mean().mul(gain).backward()

        if phase in ['Dmain', 'Dreg', 'Dboth']:
            name = 'Dreal' if phase == 'Dmain' else 'Dr1' if phase == 'Dreg' else 'Dreal_Dr1'
            with torch.autograd.profiler.record_function(name + '_forward'):
                real_tmp = real_img.detach().requires_grad_(phase in ['Dreg', 'Dboth'])
                logits = self.run_D(real_tmp, real_c, blur_sigma=blur_sigma,
                                    allow_aug_debug_print=self.allow_aug_debug_print)
                report('Loss/scores/real', logits)
                report('Loss/signs/real', logits.sign())
                loss_Dreal = 0
                if phase in ['Dmain', 'Dboth']:
                    loss_Dreal = torch.nn.functional.softplus(-logits)
                    report('Loss/D/loss', loss_Dgen + loss_Dreal)
                loss_Dr1 = 0
                if phase in ['Dreg', 'Dboth']:
                    with torch.autograd.profiler.record_function('r1_grads'), conv2d_gradfix.no_weight_gradients():
                        r1_grads = torch.autograd.grad(outputs=[logits.sum()], inputs=[real_tmp], create_graph=True,
                                                       only_inputs=True)[0]
                    r1_penalty = r1_grads.square().sum([1, 2, 3])
                    loss_Dr1 = r1_penalty * (self.r1_gamma / 2)
                    report('Loss/r1_penalty', r1_penalty)
                    report('Loss/D/reg', loss_Dr1)
            with torch.autograd.profiler.record_function(name + '_backward'):
                (loss_Dreal + loss_Dr1).mean().mul(gain).backward()
