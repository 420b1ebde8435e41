<?php

namespace Core\Processor;

use Core\Entity\Image\OutputImage;
use Core\Exception\ExecFailedException;

/**
 * Drop-in for ImageProcessor (src/Core/Processor/ImageProcessor.php) that runs
 * the resample step on an MI355X through libflyimg_hip.so over PHP FFI instead
 * of exec'ing `convert` (ImageProcessor.php:49-57, Processor.php:44-62).
 *
 * smc_1 keeps the reference's order by default: this processor resamples and
 * MozJPEG-encodes the output file, then ImageHandler::smartCropProcess
 * (ImageHandler.php:125-133) runs HipSmartCropProcessor, which takes the box
 * on the decoded output FILE -- the bytes smartcrop.py reads
 * (SmartCropProcessor.php:24) -- on the GPU and crops with `convert -crop` as
 * the reference does.  FLYIMG_HIP_FUSED_SMARTCROP=1 opts into the fused form
 * (FI_OP_SMARTCROP_APPLY: box and crop on the raw resized pixels in the same
 * call, one encode); its box differs from the reference's on ~11 % of images
 * (INTEGRATION.md).
 *
 * Geometry and option semantics are the parent's: the same OptionsBag keys,
 * the same calculateSize() decision (:115-130) and updateTargetDimensions()
 * clamp (:277-295); they are translated to one fi_image descriptor instead of
 * a command line.  Decode/encode stay on the host (djpeg -> PPM -> GPU ->
 * cjpeg, as ImageProcessor.php:204-209 pipes TGA into MozJPEG).
 * Errors raise ExecFailedException, as Processor::execute does.
 *
 * Anything the GPU path does not reproduce goes to the parent's convert
 * pipeline unchanged (gpuEligible): non-JPEG sources (PNG / GIF / WebP,
 * palette and alpha inputs), JPEGs with an EXIF orientation other than 1
 * (the parent's -auto-orient, :78), gray (1-component) JPEGs, outputs the
 * parent would not write with MozJPEG (webp / png / gif, mozjpeg off), and
 * options IM would honour or reject that the GPU path does not implement
 * (-background, colorspaces other than sRGB / RGB / Gray, gravities IM
 * does not know, non-integral -rotate).
 */
class HipImageProcessor extends ImageProcessor
{
    private const FI_OP_THUMBNAIL = 1 << 0;
    private const FI_OP_RESIZE = 1 << 1;
    private const FI_GEOM_FILL = 1 << 2;
    private const FI_GEOM_SHRINK_ONLY = 1 << 3;
    private const FI_OP_EXTENT = 1 << 4;
    private const FI_OP_GRAY = 1 << 5;
    private const FI_OP_MONOCHROME = 1 << 6;
    private const FI_OP_ROTATE = 1 << 7;
    private const FI_OP_SMARTCROP = 1 << 8;
    private const FI_OP_SMARTCROP_APPLY = 1 << 9;
    private const FI_OP_UNSHARP = 1 << 10;
    private const FI_OP_SHARPEN = 1 << 11;
    private const FI_OP_BLUR = 1 << 12;
    private const GRAVITY = ['NorthWest' => 1, 'North' => 2, 'NorthEast' => 3, 'West' => 4, 'Center' => 5,
        'East' => 6, 'SouthWest' => 7, 'South' => 8, 'SouthEast' => 9];

    /** @var \FFI|null one library handle and one fi_ctx per PHP-FPM worker */
    private static $ffi = null;
    private static $ctx = null;
    /** @var array<string, bool> output paths the fused smc_1 already cropped */
    private static $fusedCropped = [];

    /** The FFI handle and the worker's fi_ctx (shared with HipSmartCropProcessor). */
    public static function ffi(): \FFI
    {
        return self::lib();
    }

    public static function context()
    {
        self::lib();
        return self::$ctx;
    }

    /** FLYIMG_HIP_FUSED_SMARTCROP=1: box and crop inside fi_process_batch (opt-in). */
    public static function fusedSmartCrop(): bool
    {
        return getenv('FLYIMG_HIP_FUSED_SMARTCROP') === '1';
    }

    /** True once, for an output the fused smc_1 already cropped. */
    public static function takeFusedCrop(string $outputPath): bool
    {
        if (isset(self::$fusedCropped[$outputPath])) {
            unset(self::$fusedCropped[$outputPath]);
            return true;
        }
        return false;
    }

    private static function lib(): \FFI
    {
        if (self::$ffi === null) {
            $dir = getenv('FLYIMG_HIP_DIR') ?: '/opt/flyimg-hip';
            self::$ffi = \FFI::cdef(file_get_contents($dir . '/php/flyimg_hip_ffi.h'),
                $dir . '/flyimg_amd/libflyimg_hip.so');
            $ctx = self::$ffi->new('fi_ctx*');
            self::check(self::$ffi->fi_create(\FFI::addr($ctx), (int)(getenv('FLYIMG_HIP_DEVICE') ?: 0)));
            self::$ctx = $ctx;
        }
        return self::$ffi;
    }

    private static function check(int $rc): void
    {
        if ($rc !== 0) {
            throw new ExecFailedException("Command failed.\nThe exit code: " . $rc .
                "\nThe last line of output: " . self::$ffi->fi_last_error());
        }
    }

    public function processNewImage(OutputImage $outputImage): OutputImage
    {
        // a mark left by an earlier request for this path (its handler threw
        // or skipped the smart crop) must not skip this request's smart crop
        unset(self::$fusedCropped[$outputImage->getOutputImagePath()]);
        $this->sourceImageInfo = $outputImage->getInputImage()->sourceImageInfo();
        $this->options = $outputImage->getInputImage()->optionsBag();
        $path = $this->sourceImageInfo->path();
        if (!$this->gpuEligible($outputImage, $path)) {
            return parent::processNewImage($outputImage);
        }
        $decoded = self::decodeRgb($path);
        if ($decoded === null) {  // not a 3-component JPEG after all
            return parent::processNewImage($outputImage);
        }
        $ffi = self::lib();
        [$w, $h, $rgb] = $decoded;

        $img = $ffi->new('fi_image');
        $src = $ffi->new("uint8_t[" . strlen($rgb) . "]", false);
        \FFI::memcpy($src, $rgb, strlen($rgb));
        $img->src = $src;
        $img->src_w = $w;
        $img->src_h = $h;
        $img->src_stride = 3 * $w;
        $img->src_channels = 3;
        $this->describe($img, $outputImage);
        self::check($ffi->fi_plan(\FFI::addr($img), 1));
        $cap = $img->out_h * $img->out_stride;
        $dst = $ffi->new("uint8_t[$cap]", false);
        $img->dst = $dst;
        $img->dst_capacity = $cap;
        self::check($ffi->fi_process_batch(self::$ctx, \FFI::addr($img), 1));
        self::check($img->status);
        $this->encode($outputImage, \FFI::string($dst, $img->out_h * $img->out_stride),
            $img->out_w, $img->out_h, $img->out_channels);
        if ($img->flags & self::FI_OP_SMARTCROP_APPLY) {
            self::$fusedCropped[$outputImage->getOutputImagePath()] = true;
        }
        \FFI::free($src);
        \FFI::free($dst);
        return $outputImage;
    }

    /** Case-insensitive gravity lookup (IM parses -gravity case-insensitively); null = unknown. */
    private static function gravityCode(string $g): ?int
    {
        foreach (self::GRAVITY as $name => $code) {
            if (strcasecmp($name, $g) === 0) {
                return $code;
            }
        }
        return null;
    }

    /** Whether the GPU path reproduces the parent's output for this request. */
    private function gpuEligible(OutputImage $outputImage, string $path): bool
    {
        if (!is_executable(self::MOZJPEG_COMMAND) || !$outputImage->isOutputMozJpeg() ||
            $outputImage->isOutputWebP()) {
            return false;                                     // encoder choice of calculateQuality (:195-217)
        }
        $head = @file_get_contents($path, false, null, 0, 65536);
        if (!is_string($head) || strncmp($head, "\xFF\xD8\xFF", 3) !== 0) {
            return false;                                     // not a JPEG
        }
        if (self::jpegOrientation($head) > 1) {
            return false;                                     // -auto-orient would transform it
        }
        if (!empty($this->options->getOption('background'))) {
            return false;
        }
        $clsp = strtolower((string)$outputImage->extractKey('colorspace'));
        if (!in_array($clsp, ['', 'srgb', 'rgb', 'gray'], true)) {
            return false;
        }
        if (self::gravityCode((string)$this->options->getOption('gravity')) === null) {
            return false;
        }
        $rotate = (string)$this->options->getOption('rotate');
        if ($rotate !== '' && (!is_numeric($rotate) || fmod((float)$rotate, 90.0) != 0.0)) {
            return false;
        }
        return true;
    }

    /** EXIF orientation (tag 0x0112 of IFD0 in the APP1 Exif segment) of a JPEG head; 0 = none. */
    private static function jpegOrientation(string $jpg): int
    {
        $n = strlen($jpg);
        for ($p = 2; $p + 4 <= $n;) {
            if (ord($jpg[$p]) !== 0xFF) {
                return 0;
            }
            $marker = ord($jpg[$p + 1]);
            if ($marker === 0xDA || $marker === 0xD9) {
                return 0;                                     // start of scan: no Exif before it
            }
            $len = (ord($jpg[$p + 2]) << 8) | ord($jpg[$p + 3]);
            if ($marker === 0xE1 && substr($jpg, $p + 4, 6) === "Exif\0\0") {
                $t = $p + 10;                                 // TIFF header
                $le = substr($jpg, $t, 2) === 'II';
                $u16 = function (int $o) use ($jpg, $le): int {
                    $v = unpack($le ? 'v' : 'n', substr($jpg, $o, 2));
                    return $v === false ? 0 : $v[1];
                };
                $u32 = function (int $o) use ($jpg, $le): int {
                    $v = unpack($le ? 'V' : 'N', substr($jpg, $o, 4));
                    return $v === false ? 0 : $v[1];
                };
                $ifd = $t + $u32($t + 4);
                $count = $u16($ifd);
                for ($i = 0; $i < $count && $ifd + 14 + 12 * $i <= $n; $i++) {
                    $e = $ifd + 2 + 12 * $i;
                    if ($u16($e) === 0x0112) {
                        return $u16($e + 8);
                    }
                }
                return 0;
            }
            $p += 2 + $len;
        }
        return 0;
    }

    /** The fi_image equivalent of generateCommand()'s argv (:66-110). */
    private function describe($img, OutputImage $outputImage): void
    {
        $flags = empty($this->options->getOption('resize')) ? self::FI_OP_THUMBNAIL : self::FI_OP_RESIZE;
        $this->updateTargetDimensions();
        $tw = (int)$this->options->getOption('width');
        $th = (int)$this->options->getOption('height');
        if ($tw && $th && !empty($this->options->getOption('crop'))) {        // generateCropSize :138-148
            $flags |= self::FI_GEOM_FILL | self::FI_OP_EXTENT;
        } elseif ($tw || $th) {                                                 // generateSimpleSize :154-162
            if (!empty($this->options->getOption('preserve-natural-size'))) {
                $flags |= self::FI_GEOM_SHRINK_ONLY;
            }
        }
        if (strcasecmp((string)$outputImage->extractKey('colorspace'), 'Gray') === 0) {
            $flags |= self::FI_OP_GRAY;
        }
        if (!empty($outputImage->extractKey('monochrome'))) {
            $flags |= self::FI_OP_MONOCHROME;
        }
        $rotate = (int)$this->options->getOption('rotate');
        if ($rotate % 360 !== 0) {
            $flags |= self::FI_OP_ROTATE;
        }
        if (!empty($outputImage->extractKey('smart-crop')) && self::fusedSmartCrop()) {
            // opt-in fused smc_1 (ImageHandler.php:125-133 in the same call); by
            // default HipSmartCropProcessor runs on the encoded file afterwards
            $flags |= self::FI_OP_SMARTCROP | self::FI_OP_SMARTCROP_APPLY;
        }
        // forwarded -unsharp / -sharpen / -blur (:303-315), after -rotate in this order;
        // mogrify's defaults for absent geometry values: sigma 1, gain 1, threshold 0.05
        foreach (['unsharp' => [self::FI_OP_UNSHARP, [0.0, 1.0, 1.0, 0.05]],
                  'sharpen' => [self::FI_OP_SHARPEN, [0.0, 1.0]],
                  'blur' => [self::FI_OP_BLUR, [0.0, 1.0]]] as $key => [$flag, $defaults]) {
            $value = (string)$this->options->getOption($key);
            if ($value === '') {
                continue;
            }
            if (!preg_match('/^([+-]?[0-9]*\.?[0-9]+)(?:[xX,\/]([+-]?[0-9]*\.?[0-9]+))?' .
                '([+-][0-9]*\.?[0-9]+)?([+-][0-9]*\.?[0-9]+)?$/', $value, $m)) {
                throw new ExecFailedException("Command failed.\nThe exit code: geometry\nThe last line of output: " . $value);
            }
            $flags |= $flag;
            foreach ($defaults as $k => $d) {
                $img->{$key}[$k] = (isset($m[$k + 1]) && $m[$k + 1] !== '') ? (float)$m[$k + 1] : $d;
            }
        }
        $img->target_w = $tw;
        $img->target_h = $th;
        $img->flags = $flags;
        $img->gravity = self::gravityCode((string)$this->options->getOption('gravity')) ?? 5;
        $img->rotate = $rotate;
        $img->smartcrop_w = 100;                                                // smartcrop.py CLI defaults
        $img->smartcrop_h = 100;
    }

    /** Host decode to packed RGB8 (libjpeg-turbo's djpeg, PPM output); null for a
     *  gray JPEG (PGM: IM reads it as a PseudoClass image -- the parent handles it). */
    public static function decodeRgb(string $path): ?array
    {
        $ppm = shell_exec('/opt/mozjpeg/bin/djpeg -pnm ' . escapeshellarg($path));
        if (is_string($ppm) && strncmp($ppm, 'P5', 2) === 0) {
            return null;
        }
        if (!is_string($ppm) || !preg_match('/^P6\s+(\d+)\s+(\d+)\s+255\s/', $ppm, $m)) {
            throw new ExecFailedException("Command failed.\nThe exit code: decode\nThe last line of output: " . $path);
        }
        return [(int)$m[1], (int)$m[2], substr($ppm, strlen($m[0]))];
    }

    /** Host encode with MozJPEG (ImageProcessor.php:204-209 pipes TGA; PPM is equivalent). */
    private function encode(OutputImage $outputImage, string $pixels, int $w, int $h, int $c): void
    {
        $header = ($c === 1 ? "P5\n" : "P6\n") . "$w $h\n255\n";
        $cmd = escapeshellarg(self::MOZJPEG_COMMAND) . ' -quality ' .
            escapeshellarg($outputImage->extractKey('quality')) . ' -outfile ' .
            escapeshellarg($outputImage->getOutputImagePath());
        $p = proc_open($cmd, [0 => ['pipe', 'r'], 1 => ['pipe', 'w'], 2 => ['pipe', 'w']], $pipes);
        fwrite($pipes[0], $header . $pixels);
        fclose($pipes[0]);
        $err = stream_get_contents($pipes[2]);
        if (proc_close($p) !== 0) {
            throw new ExecFailedException("Command failed.\nThe exit code: encode\nThe last line of output: " . $err);
        }
    }
}
