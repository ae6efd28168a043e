"""Stride-free 3-D ResNet comparison baseline (reference
models/nostridetv_cc_smallest.py; registry name 'nostride_video_cc_small').

Stock PyTorch (Conv3d / BatchNorm3d on MIOpen): the MFMA-heavy feedforward
contrast of BASELINE.json configs[4].  Same factory
``r3d_18(pretrained=False, progress=True, **kwargs)``, module names (state_dict
keys), init and forward as the reference:

  stem: Conv3d 3->32, k (3,7,7), pad (1,3,3), no bias -> BN3d -> ReLU
  4 layers x 2 BasicBlocks, 32 channels, stride 1 everywhere, each block
      conv3x3x3-BN-ReLU -> conv3x3x3-BN, + identity, ReLU
  head: last frame of the features ++ x[:, 2, 0] (33 ch) -> Conv2d 5x5 -> 1 ch
        -> flatten (32 x 32 = 1024) -> Linear(1024, 1); returns (logits, 0).
Pretrained weights are a download (torch.hub) and are not available offline.
"""
import torch
from torch import nn

__all__ = ['VideoResNet', 'r3d_18']


class Conv3DSimple(nn.Conv3d):
    def __init__(self, in_planes, out_planes, midplanes=None, stride=1, padding=1):
        super().__init__(in_planes, out_planes, kernel_size=(3, 3, 3), stride=stride,
                         padding=padding, bias=False)

    @staticmethod
    def get_downsample_stride(stride):
        return (stride, stride, stride)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, conv_builder, stride=1, downsample=None):
        super().__init__()
        midplanes = (inplanes * planes * 27) // (inplanes * 9 + 3 * planes)
        self.conv1 = nn.Sequential(conv_builder(inplanes, planes, midplanes, 1),
                                   nn.BatchNorm3d(planes), nn.ReLU(inplace=True))
        self.conv2 = nn.Sequential(conv_builder(planes, planes, midplanes), nn.BatchNorm3d(planes))
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = 1

    def forward(self, x):
        res = x if self.downsample is None else self.downsample(x)
        return self.relu(self.conv2(self.conv1(x)) + res)


class BasicStem(nn.Sequential):
    def __init__(self):
        super().__init__(
            nn.Conv3d(3, 32, kernel_size=(3, 7, 7), stride=(1, 1, 1), padding=(1, 3, 3), bias=False),
            nn.BatchNorm3d(32),
            nn.ReLU(inplace=True))


class VideoResNet(nn.Module):
    def __init__(self, block, conv_makers, layers, stem, num_classes=1, fac=2, timesteps=None,
                 zero_init_residual=False):
        super().__init__()
        self.inplanes = 32
        self.stem = stem()
        self.layer1 = self._make_layer(block, conv_makers[0], 32, layers[0])
        self.layer2 = self._make_layer(block, conv_makers[1], 32, layers[1])
        self.layer3 = self._make_layer(block, conv_makers[2], 32, layers[2])
        self.layer4 = self._make_layer(block, conv_makers[3], 32, layers[3])
        self.avgpool = nn.AdaptiveAvgPool3d((1, 32, 32))       # registered, unused (as the reference)
        self.target_conv = nn.Conv2d(33, 1, 5, padding=2)
        nn.init.zeros_(self.target_conv.bias)
        self.fc = nn.Linear(1024, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, conv_builder, planes, blocks):
        # stride 1 and 32 -> 32 channels everywhere: no downsample branch
        layers = [block(self.inplanes, planes, conv_builder)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, conv_builder) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        target = x[:, 2, 0][:, None].clone()
        x = self.layer4(self.layer3(self.layer2(self.layer1(self.stem(x)))))
        x = self.target_conv(torch.cat([x[:, :, -1], target], 1))
        x = self.fc(x.view([int(x.shape[0]), -1]))
        return x, torch.zeros(1, device=x.device)


def r3d_18(pretrained=False, progress=True, **kwargs):
    if pretrained:
        raise NotImplementedError("pretrained weights need a download (torch.hub); offline here")
    return VideoResNet(block=BasicBlock, conv_makers=[Conv3DSimple] * 4, layers=[2, 2, 2, 2],
                       stem=BasicStem, **kwargs)
