<?php

namespace Core\Processor;

use Core\Entity\Command;
use Core\Entity\Image\OutputImage;

/**
 * Drop-in for SmartCropProcessor (src/Core/Processor/SmartCropProcessor.php:21-36)
 * that takes the smart-crop box on an MI355X over PHP FFI (fi_smartcrop) instead
 * of exec'ing `python smartcrop.py <output file>`, in the reference's order:
 *
 *   1. decode the output file HipImageProcessor (or the parent's convert) wrote
 *      -- the same bytes smartcrop.py's Image.open() reads (djpeg and Pillow
 *      are both libjpeg-turbo: islow IDCT, fancy upsampling);
 *   2. SmartCrop().crop(image, 100, 100) (smartcrop.py:359-366) as fi_smartcrop,
 *      bit-exact with smartcrop.py;
 *   3. the CLI's geometry line, "%dx%d+%d+%d" % (width + x, height + y, x, y)
 *      (smartcrop.py:368-374);
 *   4. `convert <out> -crop <geometry> <out>`, unchanged (:28-34).
 *
 * Outputs it cannot decode as 3-component JPEG (PNG / WebP / gray JPEG: the
 * mode conversions of smartcrop.py:355-363) go to the parent, i.e. the
 * SMARTCROP_COMMAND exec (the drop-in CLI `python3 -m flyimg_amd.smartcrop`).
 * An output the opt-in fused smc_1 already cropped is left as it is.
 */
class HipSmartCropProcessor extends SmartCropProcessor
{
    public function smartCrop(OutputImage $outputImage)
    {
        $path = $outputImage->getOutputImagePath();
        if (HipImageProcessor::takeFusedCrop($path)) {
            return;
        }
        $head = @file_get_contents($path, false, null, 0, 3);
        $decoded = ($head === "\xFF\xD8\xFF") ? HipImageProcessor::decodeRgb($path) : null;
        if ($decoded === null) {
            parent::smartCrop($outputImage);
            return;
        }
        [$w, $h, $rgb] = $decoded;
        $ffi = HipImageProcessor::ffi();
        $src = $ffi->new("uint8_t[" . strlen($rgb) . "]", false);
        \FFI::memcpy($src, $rgb, strlen($rgb));
        $params = $ffi->new('fi_smartcrop_params');
        $ffi->fi_smartcrop_default_params(\FFI::addr($params));
        $xywh = $ffi->new('int32_t[4]');
        $score = $ffi->new('double');
        $rc = $ffi->fi_smartcrop(HipImageProcessor::context(), $src, $w, $h, 3 * $w, 100, 100,
            \FFI::addr($params), $xywh, \FFI::addr($score));
        \FFI::free($src);
        if ($rc !== 0) {
            // smartcrop.py exits non-zero (no crop windows, ValueError): execute() throws
            throw new \Core\Exception\ExecFailedException("Command failed.\nThe exit code: " . $rc .
                "\nThe last line of output: " . $ffi->fi_last_error());
        }
        $geometry = sprintf('%dx%d+%d+%d', $xywh[2] + $xywh[0], $xywh[3] + $xywh[1], $xywh[0], $xywh[1]);
        $cropCmd = new Command(self::IM_CONVERT_COMMAND);
        $cropCmd->addArgument($path);
        $cropCmd->addArgument("-crop", $geometry);
        $cropCmd->addArgument($path);
        $this->execute($cropCmd);
    }
}
