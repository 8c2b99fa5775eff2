{{/*
Naming: the release name alone when it already mentions the chart
("gfd-amd" installed as "gfd-amd"), else "<release>-<chart>"; always a valid
63-character DNS label.
*/}}
{{- define "gfd-amd.name" -}}
{{- .Values.nameOverride | default .Chart.Name | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "gfd-amd.fullname" -}}
{{- $base := include "gfd-amd.name" . -}}
{{- $full := .Values.fullnameOverride -}}
{{- if not $full -}}
{{- $full = ternary .Release.Name (printf "%s-%s" .Release.Name $base) (contains $base .Release.Name) -}}
{{- end -}}
{{- $full | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{/* Pod labels; also the DaemonSet selector unless selectorLabelsOverride is set. */}}
{{- define "gfd-amd.podLabels" -}}
app.kubernetes.io/name: {{ include "gfd-amd.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/component: labeler
{{- end -}}

{{- define "gfd-amd.selector" -}}
{{- with .Values.selectorLabelsOverride -}}
{{ toYaml . }}
{{- else -}}
{{ include "gfd-amd.podLabels" . }}
{{- end -}}
{{- end -}}

{{/* Object labels: pod labels plus chart / version / manager. */}}
{{- define "gfd-amd.labels" -}}
{{ include "gfd-amd.podLabels" . }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name (.Chart.Version | replace "+" "_") | trunc 63 }}
{{- end -}}

{{/* Image reference; the tag defaults to v<appVersion> (versions.mk). */}}
{{- define "gfd-amd.image" -}}
{{- printf "%s:%s" .Values.image.repository (.Values.image.tag | default (printf "v%s" .Chart.AppVersion)) -}}
{{- end -}}

{{/*
Daemon flags as GFD_* environment variables, one per value that is set
(null / empty values leave the daemon's default in place).
*/}}
{{- define "gfd-amd.env" -}}
{{- $flags := dict
      "GFD_FAIL_ON_INIT_ERROR" .Values.failOnInitError
      "GFD_MIG_STRATEGY" .Values.migStrategy
      "GFD_NO_TIMESTAMP" .Values.noTimestamp
      "GFD_SLEEP_INTERVAL" .Values.sleepInterval
      "GFD_BACKEND" .Values.backend
      "GFD_AMDSMI_SESSION" .Values.amdsmiSession -}}
{{- range $name := keys $flags | sortAlpha }}
{{- $v := get $flags $name }}
{{- if not (kindIs "invalid" $v) }}
{{- if ne (toString $v) "" }}
- name: {{ $name }}
  value: {{ toString $v | quote }}
{{- end }}
{{- end }}
{{- end }}
{{- if .Values.config }}
- name: GFD_CONFIG_FILE
  value: /etc/gfd/config.yaml
{{- end }}
{{- if .Values.hostOpt.enabled }}
- name: GFD_HOST_ROOT
  value: /host
{{- end }}
{{- end -}}
