"""Results I/O in the reference's formats.

The reference's batch driver writes (speech_enhancement_comparison.py):
  - per (pair, algorithm) a result row (run_algorithm_on_pair :314-338)
    appended to summary/all_results.json (:448-451);
  - per algorithm means in summary/summary_means.json (_compute_and_save_summary
    :341-373);
  - summary/all_results.csv with a fixed header and "NA" for missing values
    (:462-471, _fmt :273-276);
  - the three optimised waveforms per (pair, algorithm) as
    {stem}_{alg}_optimized_{stoi,pesq,balanced}.wav (:302-312; soundfile's
    default WAV subtype, PCM_16).

The device scores STOI (pystoi 0.4.1 restated, metrics.py) and SNR; the pesq
extension is not in this image, so the PESQ fields are None
("NA" in the CSV), and so is everything the balance objective
(calculate_combined_speech_score of STOI and PESQ) selects: snr_balopt,
stoi_balopt, pesq_balopt, best_params_balanced stay None/{} — every reference
key keeps the reference's meaning.  The STOI-optimal cell fills the `*_stoiopt`
STOI/SNR columns and `best_params_stoi`.  The SNR-optimal cell, which the
reference does not select, is reported under keys of its own: snr_snropt and
best_params_snr (and snr_snropt_mean in summary_means.json).
"""

import json
import os
import wave

import numpy as np

ROW_KEYS = ("alg", "stem", "sr",
            "stoi_noisy", "pesq_noisy", "snr_noisy",
            "stoi_stoiopt", "pesq_stoiopt", "snr_stoiopt",
            "stoi_pesqopt", "pesq_pesqopt", "snr_pesqopt",
            "stoi_balopt", "pesq_balopt", "snr_balopt",
            "best_params_stoi", "best_params_pesq", "best_params_balanced")
CSV_HEADER = ["stem", "alg", "stoi_noisy", "pesq_noisy", "stoi_stoiopt", "pesq_stoiopt",
              "stoi_pesqopt", "pesq_pesqopt", "stoi_balopt", "pesq_balopt", "snr_balopt"]
SUMMARY_KEYS = (("stoi_noisy_mean", "stoi_noisy"), ("pesq_noisy_mean", "pesq_noisy"),
                ("stoi_stoiopt_mean", "stoi_stoiopt"), ("pesq_stoiopt_mean", "pesq_stoiopt"),
                ("stoi_pesqopt_mean", "stoi_pesqopt"), ("pesq_pesqopt_mean", "pesq_pesqopt"),
                ("stoi_balopt_mean", "stoi_balopt"), ("pesq_balopt_mean", "pesq_balopt"),
                ("snr_balopt_mean", "snr_balopt"), ("snr_snropt_mean", "snr_snropt"))


def result_row(stem, alg, sr, snr_noisy, best_snr, best_params, stoi_noisy=None,
               stoi_best=None, stoi_params=None, snr_stoiopt=None):
    """One all_results.json row (run_algorithm_on_pair :314-338).  STOI
    fields come from the device STOI (the STOI-optimal cell fills
    stoi_stoiopt / snr_stoiopt / best_params_stoi); PESQ fields are None (no
    pesq extension), and so are the PESQ-opt and balance-opt columns
    (:320-333: the balance objective needs PESQ).  The SNR-optimal cell goes
    to the extra keys snr_snropt / best_params_snr only."""
    row = {k: None for k in ROW_KEYS}
    row.update(alg=alg, stem=stem, sr=int(sr), snr_noisy=snr_noisy,
               best_params_stoi=dict(stoi_params or {}), best_params_pesq={},
               best_params_balanced={}, snr_snropt=best_snr,
               best_params_snr=dict(best_params or {}),
               stoi_noisy=stoi_noisy, stoi_stoiopt=stoi_best, snr_stoiopt=snr_stoiopt)
    return row


def fmt(x, digits=4):
    """_fmt (:267-270): 'NA' for None."""
    return "NA" if x is None else f"{x:.{digits}f}"


def summary_means(all_results, algorithms):
    """_compute_and_save_summary (:341-373) without the file write."""
    def safe_mean(values):
        valid = [v for v in values if v is not None]
        return float(np.mean(valid)) if valid else None
    out = {}
    for alg in algorithms:
        rows = [r for r in all_results if r["alg"] == alg]
        entry = {"count": len(rows)}
        for key, field in SUMMARY_KEYS:
            entry[key] = safe_mean([r.get(field) for r in rows])
        out[alg] = entry
    return out


def write_summary(all_results, algorithms, summary_dir):
    """all_results.json, summary_means.json and all_results.csv like main()."""
    os.makedirs(summary_dir, exist_ok=True)
    with open(os.path.join(summary_dir, "all_results.json"), "w", encoding="utf-8") as f:
        json.dump(all_results, f, indent=2, ensure_ascii=False)
    summary = summary_means(all_results, algorithms)
    with open(os.path.join(summary_dir, "summary_means.json"), "w", encoding="utf-8") as f:
        json.dump(summary, f, indent=2, ensure_ascii=False)
    with open(os.path.join(summary_dir, "all_results.csv"), "w", encoding="utf-8") as f:
        f.write(",".join(CSV_HEADER) + "\n")
        for r in all_results:
            row = [r["stem"], r["alg"], fmt(r["stoi_noisy"]), fmt(r["pesq_noisy"]),
                   fmt(r["stoi_stoiopt"]), fmt(r["pesq_stoiopt"]), fmt(r["stoi_pesqopt"]),
                   fmt(r["pesq_pesqopt"]), fmt(r.get("stoi_balopt")), fmt(r.get("pesq_balopt")),
                   fmt(r.get("snr_balopt"))]
            f.write(",".join(row) + "\n")
    return summary


def write_wav_pcm16(path, x, sr):
    """soundfile.write(path, float32 x, sr) with the WAV default subtype
    PCM_16, mono 16-bit little-endian.  libsndfile's float -> short write
    scales by 0x7FFF and rounds to nearest (pcm.c f2s, restated: libsndfile is
    not in this image, so this is unpinned); reads scale by 1/0x8000."""
    x = np.asarray(x, dtype=np.float32).astype(np.float64)
    q = np.clip(np.rint(x * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(q.tobytes())


def read_wav_pcm16(path):
    """(float64 samples in [-1, 1), sr) of a mono PCM16 WAV."""
    with wave.open(path, "rb") as w:
        sr = w.getframerate()
        n = w.getnframes()
        ch = w.getnchannels()
        data = np.frombuffer(w.readframes(n), dtype="<i2").astype(np.float64) / 32768.0
    if ch > 1:
        data = data.reshape(-1, ch).mean(axis=1)
    return data, sr


def shift_and_fit(y, lag, length):
    """finalize_enhanced's shift_by_lag + match_length + clip
    (speech_enhancement_comparison.py:61-69, 95-105) for writing a selected
    waveform (the device path scores it without materialising it)."""
    y = np.asarray(y, dtype=np.float64)
    if lag > 0:
        y = np.concatenate([np.zeros(lag), y])
    elif lag < 0:
        y = y[-lag:]
    if len(y) > length:
        y = y[:length]
    elif len(y) < length:
        y = np.concatenate([y, np.zeros(length - len(y))])
    return np.clip(y, -1.0, 1.0)
