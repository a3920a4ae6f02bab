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
from torch_utils.ops.staged_sum import staged_sum
from torch_utils.ops import upfirdn2d
from training.networks_stylegan2 import MinibatchStdLayer


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

    # Which terms a phase evaluates (reference loss.py:64-139): G non-saturating loss, G path-length
    # regulariser, D loss on generated images, D loss and/or R1 on real images.  A phase whose
    # regulariser weight is zero degenerates as in the reference (:66-69).
    _TERMS = {'Gmain': ('G',), 'Greg': ('Gpl',), 'Gboth': ('G', 'Gpl'),
              'Dmain': ('Dfake', 'Dreal'), 'Dreg': ('Dr1',), 'Dboth': ('Dfake', 'Dreal', 'Dr1')}

    def accumulate_gradients(self, phase, real_img, real_c, gen_z, gen_c, gain, cur_nimg):
        assert phase in self._TERMS
        terms = set(self._TERMS[phase])
        if self.pl_weight == 0:
            terms.discard('Gpl')
        if self.r1_gamma == 0:
            terms.discard('Dr1')
        sigma = 0
        if self.blur_fade_kimg > 0:
            sigma = self.blur_init_sigma * max(1 - cur_nimg / (self.blur_fade_kimg * 1e3), 0)
        # The order below is the reference's: it fixes the RNG draw sequence and the stats order.
        if 'G' in terms:
            self._generator_term(gen_z, gen_c, gain, sigma)
        if 'Gpl' in terms:
            self._path_length_term(gen_z, gen_c, gain)
        if terms == {'Dfake', 'Dreal'} and self._d_batchable(gen_z.shape[0] + real_img.shape[0]):
            self._discriminator_main_batched(real_img, real_c, gen_z, gen_c, gain, sigma)
            return
        fake_loss = self._discriminator_fake_term(gen_z, gen_c, gain, sigma) if 'Dfake' in terms else 0
        if 'Dreal' in terms or 'Dr1' in terms:
            self._discriminator_real_term(real_img, real_c, gain, sigma, fake_loss,
                                          main='Dreal' in terms, r1='Dr1' in terms)

    # Dmain's two D passes (generated, real) run as ONE forward + backward over the concatenated batch: D is
    # per-sample except the minibatch-std layer, which takes its statistics within each half
    # (MinibatchStdLayer.segments).  Same terms, same RNG draws in the same order (G, augment(fake),
    # augment(real); D draws nothing), gradients equal up to f32 summation order; half the launches.
    batch_d_main = True

    def _d_batchable(self, n):
        """Batch Dmain only when every minibatch-std layer of D can take per-segment statistics and the
        largest D activation of the combined batch `n` stays within the kernels' 32-bit byte offsets."""
        if not self.batch_d_main:
            return False
        cached = getattr(self, '_d_bytes', None)
        if cached is None or cached[0] is not self.D:
            mb = [m for m in self.D.modules() if type(m).__name__ == 'MinibatchStdLayer']
            per_sample = 0 if all(isinstance(m, MinibatchStdLayer) for m in mb) else None
            for m in self.D.modules():
                if per_sample is not None and all(hasattr(m, k) for k in ('resolution', 'in_channels', 'use_fp16', 'conv0')):
                    ch = max(m.in_channels, m.conv0.in_channels, m.conv0.out_channels)
                    per_sample = max(per_sample, ch * (m.resolution + 3) ** 2 * 4)   # the ABI's size check: 4 B/elt
            cached = self._d_bytes = (self.D, per_sample)
        return cached[1] is not None and n * cached[1] < (1 << 31) - (1 << 26)

    def backward_passes(self, phase, n=None):
        """How many backward passes of `phase` accumulate into each parameter (GradExchange hooks); `n` is
        the combined Dmain batch (generated + real)."""
        if phase == 'Dboth' or (phase == 'Dmain' and not (n is not None and self._d_batchable(n))):
            return 2
        return 1

    def _d_input(self, img, sigma, allow_aug_debug_print=False):
        """run_D without D: blur and augment (loss.py:54-60)."""
        blur_size = np.floor(sigma * 3)
        if blur_size > 0:
            with torch.autograd.profiler.record_function('blur'):
                f = torch.arange(-blur_size, blur_size + 1, device=img.device).div(sigma).square().neg().exp2()
                img = upfirdn2d.filter2d(img, f / f.sum())
        if self.augment_pipe is not None:
            img = self.augment_pipe(img, allow_aug_debug_print)
        return img

    def _discriminator_main_batched(self, real, real_c, z, c, gain, sigma):
        with torch.autograd.profiler.record_function('D_main'):
            img, _ = self.run_G(z, c, update_emas=True)
            x_fake = self._d_input(img, sigma)
            x_real = self._d_input(real.detach(), sigma, allow_aug_debug_print=self.allow_aug_debug_print)
            n = x_fake.shape[0]
            mbstd = [m for m in self.D.modules() if isinstance(m, MinibatchStdLayer)]
            for m in mbstd:
                m.segments = (n, x_real.shape[0])
            try:
                logits = self.D(torch.cat([x_fake, x_real]), torch.cat([c, real_c]), update_emas=True)
            finally:
                for m in mbstd:
                    m.segments = None
            lf, lr = logits[:n], logits[n:]
            self._report_logits('fake', lf)
            self._report_logits('real', lr)
            fake_term = torch.nn.functional.softplus(lf)
            real_term = torch.nn.functional.softplus(-lr)
            training_stats.report('Loss/D/loss', fake_term + real_term)
            (fake_term.mean() + real_term.mean()).mul(gain).backward()

    def _report_logits(self, kind, logits):
        training_stats.report(f'Loss/scores/{kind}', logits)
        training_stats.report_sign(f'Loss/signs/{kind}', logits)

    def _generator_term(self, z, c, gain, sigma):
        """-log sigmoid(D(G(z))) on a full batch (reference :73-82)."""
        with torch.autograd.profiler.record_function('G_nonsat'):
            img, _ = self.run_G(z, c)
            logits = self.run_D(img, c, blur_sigma=sigma)
            self._report_logits('fake', logits)
            term = torch.nn.functional.softplus(-logits)
            training_stats.report('Loss/G/loss', term)
            term.mean().mul(gain).backward()

    def _path_length_term(self, z, c, gain):
        """Path-length penalty pl_weight * (|J^T y| - a)^2 on 1/pl_batch_shrink of the batch, y ~ N(0, 1/HW)
        per pixel, a the running mean of |J^T y| (reference :85-100).  J^T y is a create_graph VJP through
        the synthesis network; inside no_weight_gradients the weight-gradient kernels are skipped."""
        with torch.autograd.profiler.record_function('G_path_length'):
            n = z.shape[0] // self.pl_batch_shrink
            img, ws = self.run_G(z[:n], c[:n])
            y = torch.randn_like(img) / np.sqrt(img.shape[2] * img.shape[3])
            with conv2d_gradfix.no_weight_gradients(self.pl_no_weight_grad):
                # staged: torch's split form of this 1M-value sum issues a memset into the phase graph (staged_sum.py)
                jty, = torch.autograd.grad(outputs=[staged_sum(img * y, range(img.ndim))], inputs=[ws],
                                           create_graph=True, only_inputs=True)
            lengths = jty.square().sum(2).mean(1).sqrt()
            a = self.pl_mean.lerp(lengths.mean(), self.pl_decay)
            self.pl_mean.copy_(a.detach())
            penalty = (lengths - a).square()
            training_stats.report('Loss/pl_penalty', penalty)
            term = penalty * self.pl_weight
            training_stats.report('Loss/G/reg', term)
            term.mean().mul(gain).backward()

    def _discriminator_fake_term(self, z, c, gain, sigma):
        """-log(1 - sigmoid(D(G(z)))), with the mapping / D EMAs updated (reference :104-112).  Returns the
        per-sample term for the D loss statistic."""
        with torch.autograd.profiler.record_function('D_fake'):
            img, _ = self.run_G(z, c, update_emas=True)
            logits = self.run_D(img, c, blur_sigma=sigma, update_emas=True)
            self._report_logits('fake', logits)
            term = torch.nn.functional.softplus(logits)
            term.mean().mul(gain).backward()
        return term

    def _discriminator_real_term(self, real, c, gain, sigma, fake_loss, main, r1):
        """-log sigmoid(D(x)) and/or the R1 penalty gamma/2 * |d D(x) / dx|^2 on reals, one backward
        (reference :116-139).  The R1 gradient is a create_graph VJP back through D and the ADA pipe."""
        with torch.autograd.profiler.record_function('D_real'):
            x = real.detach().requires_grad_(r1)
            logits = self.run_D(x, c, blur_sigma=sigma, allow_aug_debug_print=self.allow_aug_debug_print)
            self._report_logits('real', logits)
            total = 0
            if main:
                term = torch.nn.functional.softplus(-logits)
                training_stats.report('Loss/D/loss', fake_loss + term)
                total = term
            if r1:
                with conv2d_gradfix.no_weight_gradients():
                    gx, = torch.autograd.grad(outputs=[logits.sum()], inputs=[x], create_graph=True, only_inputs=True)
                penalty = gx.square().sum([1, 2, 3])
                reg = penalty * (self.r1_gamma / 2)
                training_stats.report('Loss/r1_penalty', penalty)
                training_stats.report('Loss/D/reg', reg)
                total = total + reg
            total.mean().mul(gain).backward()
